// compat_demod.hip -- SignalProcessor.process on gfx950, bit-compatible with the reference.
//
// Reference path (/root/reference/tetraear/signal/processor.py:221-273):
//   scipy.signal.decimate(x, q)      cheby1(8,0.05,0.8/q) SOS, sosfiltfilt (odd pad 27)   :254
//   frequency_shift                   x * exp(-j*2*pi*f*n/fs)                              :85-100
//   filter_signal                     butter(4) + filtfilt (odd pad 15), complex128        :51-83
//   extract_symbols                   best integer phase by mean |x|^2, then gather       :168-219
//   demodulate_dqpsk                  normalise, differential phase, shifted thresholds   :102-166
//
// Numerics: every recursion restates the operation order of scipy's compiled loops (no FMA
// contraction: built with -ffp-contract=off), and the vector math follows numpy's kernels on
// x86-64 (complex multiply fma(a,c,-(b*d)) / fma(a,d,b*c); |z| = max*sqrt(fma(r,r,1)),
// pairwise summation for np.mean).  Only sin/cos (mixer) and atan2 (decision) come from a
// different libm, i.e. they can differ from the CPU by an ulp.
//
// Parallel layout: IIR recursions are sequential in time, so one lane owns one real component
// of one channel ("lane = (channel, re|im)"); channels batch across lanes.  Per-lane streams
// live in a "grouped" layout [C/32][time][32 channels][re,im] so the 64 lanes of a wave touch
// 64 consecutive scalars per time step (coalesced).
#include "common.h"

namespace {

// Strided view of complex rows: element (ch, n) real part at base[off(ch, n)], imag at +1.
struct Lay {
    size_t s_grp, s_n, s_lane;
    __host__ __device__ size_t off(int ch, long n) const {
        return (size_t)(ch >> 5) * s_grp + (size_t)n * s_n + (size_t)(ch & 31) * s_lane;
    }
};
static Lay row_major(long len) { return Lay{(size_t)64 * len, 2, (size_t)2 * len}; }
static Lay grouped(long len) { return Lay{(size_t)64 * len, 64, 2}; }
static size_t grouped_elems(int C, long len) { return (size_t)((C + 31) / 32) * 64 * (size_t)len; }

constexpr int NSEC = 4;   // decimate's cheby1(8) -> 4 second-order sections

// ------------------------------------------------------------------ decimator (sosfiltfilt)
template <typename T>
__device__ __forceinline__ T sos_step(const T (&c)[NSEC * 6], T (&z)[NSEC * 2], T xc) {
#pragma unroll
    for (int s = 0; s < NSEC; ++s) {
        // scipy _sosfilt: x_new = b0*x + z0; z0 = (b1*x - a1*x_new) + z1; z1 = b2*x - a2*x_new
        T xn = c[6 * s + 0] * xc + z[2 * s];
        z[2 * s] = (c[6 * s + 1] * xc - c[6 * s + 4] * xn) + z[2 * s + 1];
        z[2 * s + 1] = c[6 * s + 2] * xc - c[6 * s + 5] * xn;
        xc = xn;
    }
    return xc;
}

// Skewed section pipeline: lane = (channel, component, section).  The 4 sections of one stream sit
// in 4 adjacent lanes; at tick tau section s processes ext sample tau - s, and its input is the
// output section s-1 produced at tick tau-1 (one DPP row shift).  Each lane runs one biquad per
// tick, so a stream's 36-operation step becomes a 9-operation tick on 4x the lanes -- the
// arithmetic (scipy _sosfilt's operation order per section and sample) is unchanged.
template <typename T>
__device__ __forceinline__ T from_left(T v) {   // lane l receives v of lane l-1 (row shift, DPP)
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
    } else {
        const long long b = __builtin_bit_cast(long long, v);
        const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffff), 0x111, 0xf, 0xf, true);
        const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x111, 0xf, 0xf, true);
        return __builtin_bit_cast(T, ((long long)hi << 32) | (unsigned int)lo);
    }
}

template <typename T>
struct Biquad {
    T b0, b1, b2, a1, a2, z0, z1;
    __device__ __forceinline__ T step(T x) {   // scipy _sosfilt, one section
        const T xn = b0 * x + z0;
        z0 = (b1 * x - a1 * xn) + z1;
        z1 = b2 * x - a2 * xn;
        return xn;
    }
};

// fp32: the same operations, paired -- (b1 x, b2 x) and (a1 xn, a2 xn) are each one v_pk_mul_f32
// (x and xn broadcast by op_sel_hi) and the two differences one v_pk_add_f32 (the product negated
// by neg_lo/neg_hi: a - b and a + (-b) are the same IEEE operation), so a section's tick is 6 VALU
// instead of 9.  Every product and sum is the scalar one, rounded once: bit-identical.
typedef float pkf2 __attribute__((ext_vector_type(2)));
template <>
struct Biquad<float> {
    pkf2 b12, a12;
    float b0, z0, z1;
    __device__ __forceinline__ Biquad(float b0_, float b1, float b2, float a1, float a2, float z0_, float z1_)
        : b12{b1, b2}, a12{a1, a2}, b0(b0_), z0(z0_), z1(z1_) {}
    __device__ __forceinline__ float step(float x) {
        const float m0 = b0 * x;
        const pkf2 p1 = b12 * pkf2{x, x};
        const float xn = m0 + z0;
        const pkf2 p3 = p1 - a12 * pkf2{xn, xn};
        z0 = p3.x + z1;
        z1 = p3.y;
        return xn;
    }
};

template <typename T>
__device__ __forceinline__ Biquad<T> load_section(const T *sos, const T *zi, int s, T x0) {
    return Biquad<T>{sos[6 * s], sos[6 * s + 1], sos[6 * s + 2], sos[6 * s + 4], sos[6 * s + 5], zi[2 * s] * x0,
                     zi[2 * s + 1] * x0};
}

constexpr int SKB = 32;   // ticks per prefetch batch (a multiple of every vector width below)
constexpr int SOS_PD = 2;   // banked decimator passes: input batches in flight

// 16-byte vectors: the decimator's memory traffic goes through as few VMEM instructions as
// possible -- with one wave per SIMD the per-wave limit on outstanding VMEM operations, not
// bandwidth or arithmetic, sets the tick rate when every tick loads and stores.
template <typename T> struct Vec16;
template <> struct Vec16<float> { using type = float4; static constexpr int n = 4; };
template <> struct Vec16<double> { using type = double2; static constexpr int n = 2; };
template <typename V> __device__ __forceinline__ auto velt(const V &v, int i) {   // i compile-time after unroll
    if constexpr (sizeof(V) == 4 * sizeof(v.x)) return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
    else return i == 0 ? v.x : v.y;
}

// Forward pass over the odd extension ext[0, L) of one stream, L = N + 2 pad.  Scratch is
// stream-major: stream g = 2 ch + comp at scr[g * Lp + j] (Lp a multiple of 4), so a lane's
// consecutive outputs are one vector store.  Input rows are complex [C][N]; a vector load holds
// CPV consecutive complex samples of both components (CPV = 2 for complex64 rows of even length).
template <typename T, int CPV>
__global__ __launch_bounds__(256) void k_sos_fwd(const T *__restrict__ x, int C, long N, int pad,
                                                const T *__restrict__ sos, const T *__restrict__ zi,
                                                T *__restrict__ scr, long Lp) {
    using V = typename Vec16<T>::type;
    constexpr int VW = Vec16<T>::n;           // outputs per vector store
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int g = gid >> 2, sec = gid & 3;
    const int ch = min(g >> 1, C - 1), comp = g & 1;   // tail lanes shadow the last stream, store nothing
    const bool own = (g >> 1) < C;
    const bool st = own && sec == 3;
    const T *xr = x + (size_t)ch * N * 2;      // complex row
    const long L = N + 2 * pad;
    auto xat = [&](long n) { return xr[2 * n + comp]; };
    const T two = 2, x0 = xat(0), xl = xat(N - 1);
    auto ext = [&](long j) -> T {   // scipy _arraytools.odd_ext
        if (j < pad) return two * x0 - xat(pad - j);
        if (j < pad + N) return xat(j - pad);
        return two * xl - xat(N - 2 - (j - pad - N));
    };
    Biquad<T> bq = load_section(sos, zi, sec, ext(0));
    T *sp = scr + (size_t)(2 * ch + comp) * Lp;
    T y = 0;
    auto tick = [&](long tau, T xin) __attribute__((always_inline)) {
        const T left = from_left(y);
        const long j = tau - sec;
        if (j >= 0 && j < L) {
            y = bq.step(sec == 0 ? xin : left);
            if (st) sp[j] = y;
        }
    };
    long tau = 0;
    for (; tau < pad; ++tau) tick(tau, ext(tau));
    // body: section 0 reads x[tau - pad] (vector loads of CPV complex samples, double-buffered one
    // batch ahead); section 3 emits j = tau - 3, aligned to VW because pad - 3 = 24.
    using PV = typename std::conditional<CPV * 2 * sizeof(T) == 16, V,
                                         typename std::conditional<sizeof(T) == 4, float2, double2>::type>::type;
    constexpr int NL = SKB / CPV;              // input vectors per batch
    PV xa[NL], xb[NL];
    auto ld = [&](PV (&v)[NL], long t0) __attribute__((always_inline)) {
        const PV *src = reinterpret_cast<const PV *>(xr + 2 * (t0 - pad));
#pragma unroll
        for (int k = 0; k < NL; ++k) v[k] = src[k];
    };
    auto run = [&](PV (&v)[NL], long t0) __attribute__((always_inline)) {
        T o[VW];
#pragma unroll
        for (int u = 0; u < SKB; ++u) {
            const PV &pv = v[u / CPV];
            const T xin = velt(pv, 2 * (u % CPV) + comp);
            const T left = from_left(y);
            y = bq.step(sec == 0 ? xin : left);   // all sections active: pad >= 3
            o[u % VW] = y;
            if (u % VW == VW - 1) {
                V w;
                if constexpr (VW == 4) w = V{o[0], o[1], o[2], o[3]};
                else w = V{o[0], o[1]};
                if (st) *reinterpret_cast<V *>(sp + (t0 + u - 3 - (VW - 1))) = w;   // section-3 lanes only
            }
        }
    };
    if (N >= 2 * SKB) {
        ld(xa, tau);
        ld(xb, tau + SKB);
        for (; tau + 4 * SKB <= pad + N; tau += 2 * SKB) {
            run(xa, tau);
            __builtin_amdgcn_sched_barrier(0);
            ld(xa, tau + 2 * SKB);
            run(xb, tau + SKB);
            __builtin_amdgcn_sched_barrier(0);
            ld(xb, tau + 3 * SKB);
        }
        run(xa, tau);
        run(xb, tau + SKB);
        tau += 2 * SKB;
    }
    for (; tau < L + 3; ++tau) tick(tau, tau < L ? ext(tau) : T(0));
}

// Reverse pass (sosfiltfilt's second sosfilt over the time-reversed forward output), keeping
// decimate's y[::q]: output t (= ext index t + pad) when t % q == 0.
template <typename T, int QT>
__global__ __launch_bounds__(256) void k_sos_bwd(const T *__restrict__ scr, long Lp, int C, long N, int pad, int q,
                                                const T *__restrict__ sos, const T *__restrict__ zi,
                                                T *__restrict__ out, Lay lo) {
    using V = typename Vec16<T>::type;
    constexpr int VW = Vec16<T>::n;
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int g = gid >> 2, sec = gid & 3;
    const int ch = min(g >> 1, C - 1), comp = g & 1;
    const bool own = (g >> 1) < C;
    const T *sp = scr + (size_t)(2 * ch + comp) * Lp;
    const long L = N + 2 * pad;
    Biquad<T> bq = load_section(sos, zi, sec, sp[L - 1]);
    T *op = out + lo.off(ch, 0) + comp;
    const size_t so = lo.s_n;
    const bool st = own && sec == 3;
    T y = 0;
    // tick tau: section 0 reads scr[L-1-tau]; section s works on ext index j = L-1-(tau-s)
    auto tick = [&](long tau, T xin) __attribute__((always_inline)) {
        const T left = from_left(y);
        const long k = tau - sec;
        if (k >= 0 && k < L) {
            y = bq.step(sec == 0 ? xin : left);
            const int t = (int)(L - 1 - k - pad);
            if (st && t >= 0 && t < N && t % q == 0) op[(size_t)(t / q) * so] = y;
        }
    };
    long tau = 0;
    if constexpr (QT == 0) {
        // body batches start where the first vector load is aligned: (L - tau) % VW == 0, tau >= 3
        long tau0 = 3;
        while ((L - tau0) % VW) ++tau0;
        for (; tau < tau0; ++tau) tick(tau, sp[L - 1 - tau]);
        constexpr int NL = SKB / VW;
        V xa[NL], xb[NL];
        auto ld = [&](V (&v)[NL], long t0) __attribute__((always_inline)) {
            // ticks t0 .. t0+SKB-1 read j = L-1-t0 down to L-t0-SKB; vector k covers
            // [L - t0 - (k+1) VW, L - t0 - k VW)
    #pragma unroll
            for (int k = 0; k < NL; ++k) v[k] = *reinterpret_cast<const V *>(sp + (L - t0 - (k + 1) * VW));
        };
        // The output lanes' index t = L-1-(tau-3)-pad falls by one per tick and is the same for every
        // stream (equal lengths), so t / q and t % q are wave-uniform scalars: the decimating store is
        // a scalar branch, not per-lane arithmetic.
        int tc = 0, tq = 0, tr = 0;
        auto run = [&](V (&v)[NL], long t0) __attribute__((always_inline)) {
    #pragma unroll
            for (int u = 0; u < SKB; ++u) {
                const T xin = velt(v[u / VW], VW - 1 - (u % VW));
                const T left = from_left(y);
                y = bq.step(sec == 0 ? xin : left);
                if (tr == 0 && tc >= 0 && tc < N) {
                    if (st) op[(size_t)tq * so] = y;
                }
                --tc;
                if (--tr < 0) { tr = q - 1; --tq; }
            }
        };
        if (L - tau >= 2 * SKB) {
            tc = __builtin_amdgcn_readfirstlane((int)(L - 1 - (tau - 3) - pad));   // >= 0 here
            tq = __builtin_amdgcn_readfirstlane(tc / q);
            tr = __builtin_amdgcn_readfirstlane(tc % q);
            ld(xa, tau);
            ld(xb, tau + SKB);
            for (; tau + 4 * SKB <= L; tau += 2 * SKB) {
                run(xa, tau);
                __builtin_amdgcn_sched_barrier(0);
                ld(xa, tau + 2 * SKB);
                run(xb, tau + SKB);
                __builtin_amdgcn_sched_barrier(0);
                ld(xb, tau + 3 * SKB);
            }
            run(xa, tau);
            run(xb, tau + SKB);
            tau += 2 * SKB;
        }
    } else {
        // q = QT known at compile time: batches of SB ticks (a multiple of QT and of VW) that start
        // where the vector load is aligned, inside the span where every output index lies in [0, N).
        // The output phase ph (the first tick u of a batch with t % QT == 0) is then the same for
        // every batch (it cannot always be 0: with the odd pad the aligned starts have odd t), so
        // the section output of each tick goes to a register yr[u] and the batch ends with SB / QT
        // stores of yr[ph + k QT] -- no per-tick counters or branches.
        constexpr int SB = (2 * QT) % VW == 0 ? 2 * QT : 4 * QT;
        constexpr int NL = SB / VW;
        auto tcur = [&](long tt) { return L - 1 - (tt - 3) - pad; };   // output index t of section 3 at tick tt
        long tau0 = pad + 3;   // first tick whose t < N
        while ((L - tau0) % VW) ++tau0;
        const int ph = __builtin_amdgcn_readfirstlane((int)(tcur(tau0) % QT));   // t % QT == 0 at u = ph
        for (; tau < tau0; ++tau) tick(tau, sp[L - 1 - tau]);
        V xa[NL], xb[NL];
        auto ld = [&](V (&v)[NL], long t0) __attribute__((always_inline)) {
#pragma unroll
            for (int k = 0; k < NL; ++k) v[k] = *reinterpret_cast<const V *>(sp + (L - t0 - (k + 1) * VW));
        };
        T *dst0 = op;
        auto run = [&](V (&v)[NL], long t0) __attribute__((always_inline)) {
            const long tq0 = (tcur(t0) - ph) / QT;   // wave-uniform: output index of tick ph
            T yr[SB];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const T xin = velt(v[u / VW], VW - 1 - (u % VW));
                const T left = from_left(y);
                y = bq.step(sec == 0 ? xin : left);
                yr[u] = y;
            }
            if (st) {
#pragma unroll
                for (int k = 0; k < SB / QT; ++k) dst0[(size_t)(tq0 - k) * so] = yr[ph + k * QT];
            }
        };
        // batches while the last tick of the next two batches still has t >= 0 (t = tcur(tau + 2 SB - 1))
        if (tcur(tau + 2 * SB - 1) >= 0 && L - tau >= 2 * SB) {
            ld(xa, tau);
            ld(xb, tau + SB);
            for (; tcur(tau + 4 * SB - 1) >= 0 && tau + 4 * SB <= L; tau += 2 * SB) {
                run(xa, tau);
                __builtin_amdgcn_sched_barrier(0);
                ld(xa, tau + 2 * SB);
                run(xb, tau + SB);
                __builtin_amdgcn_sched_barrier(0);
                ld(xb, tau + 3 * SB);
            }
            run(xa, tau);
            run(xb, tau + SB);
            tau += 2 * SB;
        }
    }
    for (; tau < L + 3; ++tau) tick(tau, tau < L ? sp[L - 1 - tau] : T(0));
}

// ------------------------------------------------------------------ fp32 decimator, banked lanes
// The kernels above are bound by the texture data path (TD ~95 % busy, r01 PMC): the four
// section lanes of a stream, and for the forward pass both components of a channel, load the same
// 16 bytes, so every load instruction returns 1 KiB for 128-256 useful bytes.  Here the section
// is the DPP bank instead of the low lane bits:
//   lane = 16 row + 4 sec + s,   stream g = 16 wave + 4 row + s   (g = 2 ch + comp)
// The section chain moves one bank right per tick (row_shr:4), and the 4 lanes of a stream load 4
// DIFFERENT 16-byte chunks of its input window; section 0 (bank 0) takes the tick's sample from
// the lane of bank j with row_shl:4j under bank_mask 1 -- the same DPP move that replaces the
// section-0 select, so a tick is 2 DPP moves + the 9-operation biquad.  Arithmetic per section and
// sample is unchanged (bit-identical to the kernels above and to scipy's _sosfilt).
template <int CTRL, int BANKS, bool BC>
__device__ __forceinline__ float dppf(float old, float src) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                                 __builtin_bit_cast(int, src), CTRL, 0xf, BANKS, BC));
}
// section 0 takes src of bank j (compile time); the other banks keep `left`
template <int J>
__device__ __forceinline__ float bank0_from(float left, float src) {
    if constexpr (J == 0) return dppf<0xE4, 0x1, false>(left, src);   // quad_perm identity
    else return dppf<0x100 + 4 * J, 0x1, false>(left, src);            // row_shl:4J
}
__device__ __forceinline__ float from_left_bank(float y) { return dppf<0x114, 0xf, true>(0.f, y); }   // row_shr:4

// 4-byte aligned 16-byte load (the imaginary stream's window starts one float into a complex pair)
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

struct BankLane {
    int sec, g, ch, comp;
    bool own, st;
    __device__ BankLane(int C) {
        const int lane = threadIdx.x & 63, w = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
        sec = (lane >> 2) & 3;
        g = 16 * w + 4 * (lane >> 4) + (lane & 3);
        ch = min(g >> 1, C - 1);   // tail lanes shadow the last stream and store nothing
        comp = g & 1;
        own = (g >> 1) < C;
        st = own && sec == 3;
    }
};

// Forward pass (k_sos_fwd's contract) for complex64 rows of any length: the window loads are
// 4-byte-aligned vectors (f4u), so an odd-length row's 8-byte-aligned start is fine, and the
// batches stop one sample short of the row end (below).  Window of 8 samples:
// lane (sec = j) loads floats [2 n0 + 4 j + comp, +4): elements 0 and 2 are component `comp` of
// samples n0 + 2j and n0 + 2j + 1.
__global__ __launch_bounds__(256) void k_sos_fwd_bank(const float *__restrict__ x, int C, long N, int pad,
                                                     const float *__restrict__ sos, const float *__restrict__ zi,
                                                     float *__restrict__ scr, long Lp) {
    const BankLane bl(C);
    const int sec = bl.sec, comp = bl.comp;
    const bool st = bl.st;
    const float *xr = x + (size_t)bl.ch * N * 2;
    const long L = N + 2 * pad;
    auto xat = [&](long n) { return xr[2 * n + comp]; };
    const float two = 2, x0 = xat(0), xl = xat(N - 1);
    auto ext = [&](long j) -> float {   // scipy _arraytools.odd_ext
        if (j < pad) return two * x0 - xat(pad - j);
        if (j < pad + N) return xat(j - pad);
        return two * xl - xat(N - 2 - (j - pad - N));
    };
    Biquad<float> bq = load_section(sos, zi, sec, ext(0));
    float *sp = scr + (size_t)(2 * bl.ch + comp) * Lp;
    float y = 0;
    auto tick = [&](long tau, float xin) __attribute__((always_inline)) {
        const float left = from_left_bank(y);
        const long j = tau - sec;
        if (j >= 0 && j < L) {
            y = bq.step(sec == 0 ? xin : left);
            if (st) sp[j] = y;
        }
    };
    long tau = 0;
    for (; tau < pad; ++tau) tick(tau, ext(tau));
    constexpr int NW = SKB / 8;   // 8-sample windows per batch
    const float *xw = xr + 4 * sec + comp;
    auto ld = [&](f4u (&v)[NW], long t0) __attribute__((always_inline)) {
        const float *src = xw + 2 * (t0 - pad);
#pragma unroll
        for (int k = 0; k < NW; ++k) v[k] = *reinterpret_cast<const f4u *>(src + 16 * k);
    };
    // Output: section 3 emits j = tau - 3.  Every 16 ticks the four lanes of a stream each store 4
    // of section 3's last 16 outputs (bank j takes o[4j .. 4j+3] from bank 3 with row_shl:4(3-j)):
    // one 64-lane store of 64 contiguous bytes per stream instead of four 16-lane stores of 16.
    const bool own = bl.own;
    auto run = [&](f4u (&v)[NW], long t0) __attribute__((always_inline)) {
        float o[16];
#pragma unroll
        for (int u = 0; u < SKB; ++u) {
            const f4u &pv = v[u >> 3];
            const float e = (u & 1) ? pv.z : pv.x;
            const float left = from_left_bank(y);
            float xin;
            switch ((u >> 1) & 3) {
                case 0: xin = bank0_from<0>(left, e); break;
                case 1: xin = bank0_from<1>(left, e); break;
                case 2: xin = bank0_from<2>(left, e); break;
                default: xin = bank0_from<3>(left, e); break;
            }
            y = bq.step(xin);   // every section active: pad >= 3
            o[u & 15] = y;
            if ((u & 15) == 15) {
                float w[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    w[i] = o[12 + i];
                    w[i] = dppf<0x10C, 0x1, false>(w[i], o[i]);       // bank 0 <- bank 3 (row_shl:12)
                    w[i] = dppf<0x108, 0x2, false>(w[i], o[4 + i]);   // bank 1 <- bank 3 (row_shl:8)
                    w[i] = dppf<0x104, 0x4, false>(w[i], o[8 + i]);   // bank 2 <- bank 3 (row_shl:4)
                }
                if (own) *reinterpret_cast<float4 *>(sp + (t0 + u - 18 + 4 * sec)) = float4{w[0], w[1], w[2], w[3]};
            }
        }
        // elements 1 and 3 are never read: keep the whole vector live to here, or the allocator
        // reuses them as temporaries while the next window's load into them is in flight (a
        // write-after-write wait on every outstanding load)
#pragma unroll
        for (int k = 0; k < NW; ++k) asm volatile("" ::"v"(v[k]));
    };
    // the imaginary lanes of the last chunk read one float past their window: the batches stop
    // one sample short of the row end, so that float is inside the row.  SOS_PD batches in flight.
    if (N >= SOS_PD * SKB + 1) {
        f4u xs[SOS_PD][NW];
#pragma unroll
        for (int u = 0; u < SOS_PD; ++u) ld(xs[u], tau + u * SKB);
        for (; tau + 2 * SOS_PD * SKB < pad + N; tau += SOS_PD * SKB) {
#pragma unroll
            for (int u = 0; u < SOS_PD; ++u) {
                run(xs[u], tau + u * SKB);
                __builtin_amdgcn_sched_barrier(0);
                ld(xs[u], tau + (u + SOS_PD) * SKB);
            }
        }
#pragma unroll
        for (int u = 0; u < SOS_PD; ++u) run(xs[u], tau + u * SKB);
        tau += SOS_PD * SKB;
    }
    for (; tau < L + 3; ++tau) tick(tau, tau < L ? ext(tau) : 0.f);
}

// Reverse pass with decimation q = QT (k_sos_bwd<float, QT>'s contract).  The scratch row is the
// stream's own, so the 4 lanes of a stream load the 4 chunks of a 16-tick window with no
// duplication: lane (sec = j) loads floats [L - t0 - 16 k - 4 j - 4, +4), tick u of the window reads
// element 3 - (u & 3) of chunk (u >> 2) & 3.  The batch start is chosen so that the first output
// tick of every batch is the compile-time phase PH, so outputs are stored as they are produced.
template <int QT>
__global__ __launch_bounds__(256) void k_sos_bwd_bank(const float *__restrict__ scr, long Lp, int C, long N, int pad,
                                                     int q, const float *__restrict__ sos,
                                                     const float *__restrict__ zi, float *__restrict__ out, Lay lo) {
    const BankLane bl(C);
    const int sec = bl.sec;
    const bool st = bl.st;
    const float *sp = scr + (size_t)(2 * bl.ch + bl.comp) * Lp;
    const long L = N + 2 * pad;
    Biquad<float> bq = load_section(sos, zi, sec, sp[L - 1]);
    float *op = out + lo.off(bl.ch, 0) + bl.comp;
    const size_t so = lo.s_n;
    float y = 0;
    auto tick = [&](long tau, float xin) __attribute__((always_inline)) {
        const float left = from_left_bank(y);
        const long k = tau - sec;
        if (k >= 0 && k < L) {
            y = bq.step(sec == 0 ? xin : left);
            const int t = (int)(L - 1 - k - pad);
            if (st && t >= 0 && t < N && t % q == 0) op[(size_t)(t / q) * so] = y;
        }
    };
    constexpr int SB = QT * 16 / (QT % 16 == 0 ? 16 : QT % 8 == 0 ? 8 : QT % 4 == 0 ? 4 : QT % 2 == 0 ? 2 : 1);
    static_assert(SB % 16 == 0 && SB % QT == 0, "batch = lcm(16, QT)");
    constexpr int NL = SB / 16;
    // output index of section 3 at tick tt; t % QT == 0 at tick u of a batch iff u % QT == PH
    auto tcur = [&](long tt) { return L - 1 - (tt - 3) - pad; };
    // PH must match the parity that the aligned starts allow (tcur(tau0) = L - tau0 + 2 - pad with
    // L - tau0 a multiple of 4): odd for even QT and the default odd pad
    constexpr int PH = QT % 2 ? 0 : 5 % QT;
    long tau0 = pad + 3;
    while (((L - tau0) % 4 || tcur(tau0) % QT != PH) && tau0 < pad + 3 + 4 * QT) ++tau0;
    const bool phased = (L - tau0) % 4 == 0 && tcur(tau0) % QT == PH;
    long tau = 0;
    if (phased) {
        for (; tau < tau0; ++tau) tick(tau, sp[L - 1 - tau]);
        const float *sw = sp + L - 4 - 4 * sec;
        auto ld = [&](float4 (&v)[NL], long t0) __attribute__((always_inline)) {
#pragma unroll
            for (int k = 0; k < NL; ++k) v[k] = *reinterpret_cast<const float4 *>(sw - t0 - 16 * k);
        };
        auto run = [&](float4 (&v)[NL], long t0) __attribute__((always_inline)) {
            const long tq0 = tcur(t0 + PH) / QT;   // wave-uniform: output index of tick PH
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const float4 &pv = v[u >> 4];
                const int el = 3 - (u & 3);
                const float e = el == 3 ? pv.w : el == 2 ? pv.z : el == 1 ? pv.y : pv.x;
                const float left = from_left_bank(y);
                float xin;
                switch ((u >> 2) & 3) {
                    case 0: xin = bank0_from<0>(left, e); break;
                    case 1: xin = bank0_from<1>(left, e); break;
                    case 2: xin = bank0_from<2>(left, e); break;
                    default: xin = bank0_from<3>(left, e); break;
                }
                y = bq.step(xin);
                if (u % QT == PH && st) op[(size_t)(tq0 - u / QT) * so] = y;
            }
        };
        if (tcur(tau + SOS_PD * SB - 1) >= 0 && L - tau >= SOS_PD * SB) {
            float4 xs[SOS_PD][NL];
#pragma unroll
            for (int u = 0; u < SOS_PD; ++u) ld(xs[u], tau + u * SB);
            for (; tcur(tau + 2 * SOS_PD * SB - 1) >= 0 && tau + 2 * SOS_PD * SB <= L; tau += SOS_PD * SB) {
#pragma unroll
                for (int u = 0; u < SOS_PD; ++u) {
                    run(xs[u], tau + u * SB);
                    __builtin_amdgcn_sched_barrier(0);
                    ld(xs[u], tau + (u + SOS_PD) * SB);
                }
            }
#pragma unroll
            for (int u = 0; u < SOS_PD; ++u) run(xs[u], tau + u * SB);
            tau += SOS_PD * SB;
        }
    }
    for (; tau < L + 3; ++tau) tick(tau, tau < L ? sp[L - 1 - tau] : 0.f);
}

// ------------------------------------------------------------------ time-blocked decimator (latency mode)
// sosfiltfilt for a few channels, parallel in time.  A stream's
// odd extension ext[0, L) is cut into tiles of SB_B samples; one quad of lanes runs the 4-section
// cascade over one tile (the skewed section pipeline of k_sos_fwd: section s works on sample tau - s
// at tick tau), so every tile of every stream recurses at once.  Per pass (forward, then backward on
// the reversed forward output):
//   1. k_sosb_tile<.., false>: each tile from zero state -> its end state e_k (8 numbers: the two
//      DF-II-T states of 4 sections), T arithmetic;
//   2. k_sosb_scan: the true start states s_k of every tile in float64, s_{k+1} = Phi s_k + e_k with
//      Phi = A^SB_B (A: the cascade's one-sample zero-input transition), s_0 = sosfilt_zi * ext[0] as
//      the sequential pass sets it -- as an inclusive Hillis-Steele scan over the tiles with the
//      host's table Phi^(2^r) (compat_blocked_table);
//   3. k_sosb_tile<.., true>: each tile again from (T) s_k, its outputs to the scratch row (forward)
//      or decimated to `out` (backward).
// Tile 0 starts from the sequential pass's exact state, so its outputs are scipy's bit for bit;
// later tiles start from the float64-composed state instead of the state a sequential fp32
// recursion would have accumulated, so outputs differ from scipy's by the filter's fp32 noise
// (measured on the 31 reference fixtures: <= 3.4e-6 on .symbols for q <= 10, no hard decision
// changed; oracle/compat.py: decimate_blocked restates every operation and the GPU equals it bit
// for bit).  Used by tetra_demod_compat for C <= SB_MAXC channels and q <= SB_MAXQ (at q = 83 the
// cheby1 band is so narrow the noise reaches 5.7e-5), and never by the component entry point
// tetra_decimate, which stays scipy-exact.
constexpr int SB_B = 256;        // samples per tile
constexpr int SB_MAXT = 1024;    // tiles per stream (one scan workgroup): L <= 262144
constexpr int SB_NPOW = 10;      // Phi^(2^r), r < SB_NPOW: covers SB_MAXT tiles
constexpr int SB_MAXC = 64;      // channels up to which tetra_demod_compat takes this path
constexpr int SB_MAXQ = 16;      // decimation factors up to which it does
// stream-tiles per workgroup: few, so one channel's tiles spread over many CUs; SB_LT threads stage
// them (SB_B ST / SB_LT loads each), wave 0's 4 ST lanes run the recursion
template <typename T> struct SbCfg { static constexpr int ST = 16; };
constexpr int SB_LT = 256;

struct SbGeo {
    int C, Tn, pad, q;
    long N, L, Lp;
};

// stream-tile g = (ch * Tn + tile) * 2 + comp
template <typename T, bool FWD, bool FINAL>
__global__ __launch_bounds__(SB_LT) void k_sosb_tile(const T *__restrict__ x, T *__restrict__ scr, SbGeo G,
                                                                const T *__restrict__ sos,
                                                                const double *__restrict__ states,
                                                                double *__restrict__ ends, T *__restrict__ out, Lay lo) {
    constexpr int ST = SbCfg<T>::ST;
    __shared__ T buf[ST][SB_B + 1];
    __shared__ int rch[ST], rtile[ST];   // the rows' channel and tile: one division per row, not per element
    const int tid = threadIdx.x, sec = tid & 3, stl = tid >> 2;
    const long ntiles = (long)2 * G.C * G.Tn;
    const int nrow = (int)min((long)ST, ntiles - (long)blockIdx.x * ST);   // rows this workgroup owns
    if (tid < ST) {
        const int pr = (int)((((long)blockIdx.x * ST + (tid < nrow ? tid : 0))) >> 1);
        rtile[tid] = pr % G.Tn;
        rch[tid] = pr / G.Tn;
    }
    __syncthreads();
    // cooperative load of the workgroup's tiles: ext (forward) or the reversed scratch row (backward).
    // A single channel is a few workgroups, so each thread's 64 loads are what the pass waits for:
    // they go out 16 at a time (unconditional, from clamped indices), and ext's odd-extension
    // arithmetic at the row ends is applied afterwards to the raw samples it reflects.
    constexpr int PER = ST * SB_B / SB_LT, U = PER < 16 ? PER : 16;
    static_assert(PER % U == 0 && 4 * ST <= 64, "loads per thread; the recursion fits wave 0");
    auto src = [&](int i, int &r, int &j, long &e, int &ch, int &comp, bool &in) -> const T * {
        r = i / SB_B;
        j = i % SB_B;
        in = r < nrow;
        const int rr = in ? r : 0;
        comp = rr & 1;   // ST is even: row parity = stream-tile parity
        const int tile = rtile[rr];
        ch = rch[rr];
        e = (long)tile * SB_B + j;
        in = in && e < G.L;
        const long ec = in ? e : 0;
        if (FWD) {   // the sample scipy's odd_ext reflects (or copies) at ext index e
            const long n = ec < G.pad ? G.pad - ec : (ec < G.pad + G.N ? ec - G.pad : G.N - 2 - (ec - G.pad - G.N));
            return x + (size_t)ch * G.N * 2 + comp + 2 * n;
        }
        return scr + (size_t)(2 * ch + comp) * G.Lp + (G.L - 1 - ec);
    };
    for (int c0 = 0; c0 < PER; c0 += U) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int r, j, ch, comp;
            long e;
            bool in;
            v[u] = *src(tid + SB_LT * (c0 + u), r, j, e, ch, comp, in);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int r, j, ch, comp;
            long e;
            bool in;
            src(tid + SB_LT * (c0 + u), r, j, e, ch, comp, in);
            T w = in ? v[u] : (T)0;
            if (FWD && in && (e < G.pad || e >= G.pad + G.N)) {   // scipy _arraytools.odd_ext, in T
                const T *xr = x + (size_t)ch * G.N * 2 + comp;
                w = (T)2 * (e < G.pad ? xr[0] : xr[2 * (G.N - 1)]) - w;
            }
            buf[r][j] = w;
        }
    }
    __syncthreads();
    if (tid < 4 * ST) {   // wave 0: the recursion (wave-uniform branch)
    const long g = (long)blockIdx.x * ST + stl;
    const bool own = g < ntiles;
    const int tile = own ? (int)((g >> 1) % G.Tn) : 0;
    const long len = own ? min((long)SB_B, G.L - (long)tile * SB_B) : 0;
    Biquad<T> bq{sos[6 * sec], sos[6 * sec + 1], sos[6 * sec + 2], sos[6 * sec + 4], sos[6 * sec + 5], (T)0, (T)0};
    if (FINAL && own) {
        bq.z0 = (T)states[g * 8 + 2 * sec];
        bq.z1 = (T)states[g * 8 + 2 * sec + 1];
    }
    // Ticks 0-2 and SB_B..SB_B+2 are guarded (a section starts at tick sec and ends at SB_B - 1 + sec);
    // the rest are branch-free: every lane steps and (FINAL) writes its output to slot j = tick - sec
    // -- section 3 writes slot j last, and inputs of slot j were read at the top of this batch or an
    // earlier one.  The last tile of a stream (len < SB_B) steps on the zeros past its end: its end
    // state is not used (the scan reads e_k for k < Tn - 1) and its outputs past len are not stored.
    (void)len;
    T y = 0;
    for (int tau0 = 0; tau0 < SB_B; tau0 += 16) {
        T in[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) in[u] = buf[stl][tau0 + u];
        if (tau0 == 0) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const T left = from_left(y);
                const T xin = sec == 0 ? in[u] : left;
                if (u >= 3 || u >= sec) {
                    y = bq.step(xin);
                    if (FINAL) buf[stl][u - sec] = y;
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const T left = from_left(y);
                y = bq.step(sec == 0 ? in[u] : left);
                if (FINAL) buf[stl][tau0 + u - sec] = y;
            }
        }
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {   // ticks SB_B .. SB_B + 2: sections u+1 .. 3 finish
        const T left = from_left(y);
        if (sec > u) {
            y = bq.step(left);
            if (FINAL) buf[stl][SB_B + u - sec] = y;
        }
    }
    if (!FINAL && own) {
        ends[g * 8 + 2 * sec] = (double)bq.z0;
        ends[g * 8 + 2 * sec + 1] = (double)bq.z1;
    }
    }
    if (!FINAL) return;
    __syncthreads();
    for (int i = tid; i < ST * SB_B; i += SB_LT) {
        const int r = i / SB_B, j = i % SB_B;
        if (r >= nrow) continue;
        const int comp = r & 1, tl = rtile[r], ch = rch[r];
        const long e = (long)tl * SB_B + j;
        if (e >= G.L) continue;
        if (FWD) {
            scr[(size_t)(2 * ch + comp) * G.Lp + e] = buf[r][j];
        } else {   // ext index L-1-e, sample t = ext - pad; decimate keeps t % q == 0
            const long t = G.L - 1 - e - G.pad;
            if (t >= 0 && t < G.N && t % G.q == 0) out[lo.off(ch, t / G.q) + comp] = buf[r][j];
        }
    }
}

// Start states of every tile of one stream (workgroup = stream 2 ch + comp, thread = tile):
// w_0 = sosfilt_zi * ext[0] (T, as the sequential pass computes it), w_k = e_{k-1}; then for
// d = 1, 2, 4, ..: w_k += Phi^d w_{k-d} (k >= d), each product summed in j order without FMA
// (oracle/compat.py: _blocked_scan restates it).
template <typename T, bool FWD>
__global__ __launch_bounds__(1024) void k_sosb_scan(const T *__restrict__ x, const T *__restrict__ scr, SbGeo G,
                                                    const T *__restrict__ zi, const double *__restrict__ phi,
                                                    const double *__restrict__ ends, double *__restrict__ states) {
    __shared__ double w[SB_MAXT][8];
    const int k = threadIdx.x, s = blockIdx.x, ch = s >> 1, comp = s & 1;
    const bool on = k < G.Tn;
    double v[8];
    if (on) {
        if (k == 0) {
            T x0;
            if (FWD) {
                const T *xr = x + (size_t)ch * G.N * 2 + comp;
                x0 = (T)2 * xr[0] - xr[2 * G.pad];
            } else {
                x0 = scr[(size_t)s * G.Lp + G.L - 1];
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = (double)(zi[i] * x0);
        } else {
            const double *e = ends + ((size_t)(ch * G.Tn + k - 1) * 2 + comp) * 8;
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = e[i];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) w[k][i] = v[i];
    }
    for (int r = 0; (1 << r) < G.Tn; ++r) {
        const int d = 1 << r;
        __syncthreads();
        double u[8];
        const bool upd = on && k >= d;
        if (upd) {
#pragma unroll
            for (int i = 0; i < 8; ++i) u[i] = w[k - d][i];
        }
        __syncthreads();
        if (upd) {
            // the table straight from global memory at a wave-uniform address: scalar loads, SGPR
            // operands (staged in LDS, its 36 broadcast reads per level cost ~2 us per scan:
            // profiles/r05_ab_scan_sgpr.txt)
            const double *P = phi + __builtin_amdgcn_readfirstlane(r) * 64;
            // the eight rows' sums side by side (each still j-ascending, no FMA: the same bits), then
            // the new state to LDS
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = v[i] + P[i * 8 + j] * u[j];
#pragma unroll
            for (int i = 0; i < 8; ++i) w[k][i] = v[i];
        }
    }
    if (on) {
        double *o = states + ((size_t)(ch * G.Tn + k) * 2 + comp) * 8;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = v[i];
    }
}

// A (the cascade's one-sample zero-input transition, from the coefficients the kernels use, in
// double) and the table Phi^(2^r) = A^(SB_B 2^r), r < SB_NPOW, row-major 8 x 8 each; every product
// summed in k order without FMA (the oracle computes the same table the same way).
void blocked_table(const double *coef /*[24] sos rows*/, double *tab /*[SB_NPOW * 64]*/) {
    double A[64];
    for (int k = 0; k < 8; ++k) {
        double z[8] = {0}, zn[8];
        z[k] = 1.0;
        double u = 0.0;
        for (int s = 0; s < NSEC; ++s) {
            const double *c = coef + 6 * s;
            const double xn = c[0] * u + z[2 * s];
            zn[2 * s] = (c[1] * u - c[4] * xn) + z[2 * s + 1];
            zn[2 * s + 1] = c[2] * u - c[5] * xn;
            u = xn;
        }
        for (int i = 0; i < 8; ++i) A[i * 8 + k] = zn[i];
    }
    auto square = [](const double *P, double *out) {
        double t[64];
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 8; ++j) {
                double acc = 0.0;
                for (int k = 0; k < 8; ++k) acc = acc + P[i * 8 + k] * P[k * 8 + j];
                t[i * 8 + j] = acc;
            }
        for (int i = 0; i < 64; ++i) out[i] = t[i];
    };
    for (int b = 1; b < SB_B; b <<= 1) square(A, A);   // A^SB_B (SB_B a power of two)
    for (int i = 0; i < 64; ++i) tab[i] = A[i];
    for (int r = 1; r < SB_NPOW; ++r) square(tab + (r - 1) * 64, tab + r * 64);
}

// ------------------------------------------------------------------ mixer + filtfilt (lfilter)
// Value of component `comp` of (possibly frequency-shifted) sample n, in double.
__device__ __forceinline__ double mix_pair(double xr, double xi, long n, int comp, bool mix, double c, double fs) {
    if (!mix) return comp ? xi : xr;
    // numpy: t = arange/fs; arg = (-1j*2*pi*f)*t has real part 0, imag c*t; exp(arg) = (cos, sin)
    const double th = c * ((double)n / fs);
    double s, co;
    sincos(th, &s, &co);
    // numpy SIMD complex multiply: re = fma(xr, sr, -(xi*si)), im = fma(xr, si, xi*sr)
    return comp ? fma(xr, s, xi * co) : fma(xr, co, -(xi * s));
}

template <typename TIn>
__device__ __forceinline__ double mixed_val(const TIn *xp, size_t sx, long n, int comp, bool mix, double c,
                                            double fs) {
    const double xr = (double)xp[(size_t)n * sx], xi = (double)xp[(size_t)n * sx + 1];
    if (!mix) return comp ? xi : xr;
    // numpy: t = arange/fs; arg = (-1j*2*pi*f)*t has real part 0, imag c*t; exp(arg) = (cos, sin)
    const double th = c * ((double)n / fs);
    double s, co;
    sincos(th, &s, &co);
    // numpy SIMD complex multiply: re = fma(xr, sr, -(xi*si)), im = fma(xr, si, xi*sr)
    return comp ? fma(xr, s, xi * co) : fma(xr, co, -(xi * s));
}

// Odd-extended input of filtfilt at ext index j.  The extension is computed in the precision of
// the array filtfilt receives: complex128 when mixed, else the input type (complex64 from
// decimate), then promoted to double (scipy lfilter runs in complex128).
template <typename TIn>
__device__ __forceinline__ double lf_ext(const TIn *xp, size_t sx, long M, int pad, long j, int comp, bool mix,
                                         double c, double fs) {
    long n;
    int side;
    if (j < pad) { n = pad - j; side = -1; }
    else if (j < pad + M) { n = j - pad; side = 0; }
    else { n = M - 2 - (j - pad - M); side = 1; }
    if (mix) {
        const double v = mixed_val(xp, sx, n, comp, true, c, fs);
        if (side == 0) return v;
        const double e = mixed_val(xp, sx, side < 0 ? 0 : M - 1, comp, true, c, fs);
        return 2.0 * e - v;
    }
    const TIn v = xp[(size_t)n * sx + comp];
    if (side == 0) return (double)v;
    const TIn e = xp[(size_t)(side < 0 ? 0 : M - 1) * sx + comp];
    return (double)((TIn)2 * e - v);
}

constexpr int MAXTAP = 8;

// scipy lfilter (DF-II-T) with NT taps, one stream (channel x re|im) per lane, in double:
//   y = z0 + b0*x;  z_k = (z_{k+1} + x*b_{k+1}) - y*a_{k+1};  z_{NT-2} = x*b_{NT-1} - y*a_{NT-1}
template <int NT>
struct Lfilt {
    double bb[NT], aa[NT], z[NT - 1];
    __device__ __forceinline__ void init(const double *b, const double *a, const double *zi, double x0) {
#pragma unroll
        for (int k = 0; k < NT; ++k) { bb[k] = b[k]; aa[k] = a[k]; }
#pragma unroll
        for (int k = 0; k < NT - 1; ++k) z[k] = zi[k] * x0;
    }
    __device__ __forceinline__ double step(double xn) {
        const double yn = z[0] + bb[0] * xn;
#pragma unroll
        for (int k = 0; k < NT - 2; ++k) z[k] = (z[k + 1] + xn * bb[k + 1]) - yn * aa[k + 1];
        z[NT - 2] = xn * bb[NT - 1] - yn * aa[NT - 1];
        return yn;
    }
};

// The same lfilter with its four states spread over a quad of lanes (NT = 5: butter(4)): lane k holds
// z_k; per sample every lane forms y = z_0 + b0 x from quad lane 0's state (DPP broadcast), and
// z_k = (z_{k+1} + x b_{k+1}) - y a_{k+1} from lane k+1's (DPP shift; lane 3: x b_4 - y a_4).  The
// operations and their order are Lfilt's; a sample is 5 float64 operations per wave instead of 17.
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
    const long long b = __builtin_bit_cast(long long, v);
    // quad_perm writes every lane: no `old` operand to materialise
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
struct Lfilt4 {
    double b0, bk, ak, z;
    bool last;
    __device__ __forceinline__ void init(const double *b, const double *a, const double *zi, double x0) {
        const int k = threadIdx.x & 3;
        b0 = b[0];
        bk = b[k + 1];
        ak = a[k + 1];
        z = zi[k] * x0;
        last = k == 3;
    }
    __device__ __forceinline__ double step(double xn) {
        const double z0 = dpp64<0x00>(z);   // quad_perm [0,0,0,0]: lane 0's z_0
        const double zs = dpp64<0xF9>(z);   // quad_perm [1,2,3,3]: lane k+1's z_{k+1}
        const double yn = z0 + b0 * xn;
        const double t = xn * bk;
        z = (last ? t : zs + t) - yn * ak;
        return yn;
    }
};
// Lanes per stream of the filtfilt kernels: 4 (Lfilt4) for a few channels, where one wave's issue
// sets the time -- one 131072-sample chunk (C2): filtfilt 1.97 -> ~1.7 ms, process() 7.2 -> 7.0 ms --
// and 1 (Lfilt) for batches, which are bound by the load path: at 8192 channels Lfilt4's four lanes
// per stream make the two passes 1.04 + 0.75 -> 1.30 + 0.99 ms (profiles/r06_ab_compat_lf4.txt).
// TETRA_COMPAT_LF=1 / 4 forces a form (same-box A/B).
constexpr int LF4_MAXC = 64;
static int lf_lanes(int C) {
    const char *e = getenv("TETRA_COMPAT_LF");
    if (e && (atoi(e) == 1 || atoi(e) == 4)) return atoi(e);
    return C <= LF4_MAXC ? 4 : 1;
}

constexpr int LFB = 16;   // samples per load batch; batches double-buffered

// Forward pass over the odd extension (filtfilt padlen 3*NT) of the (optionally mixed) input.
// MIX = false (launched when no channel mixes, e.g. on k_mix's pre-mixed rows): the mixer's sincos
// code leaves the loop -- with it inlined 16 times the kernel holds values in AGPRs across the
// recursion; the same operations otherwise.
// QL lanes per stream: 1 (Lfilt) or 4 (Lfilt4, NT = 5: the quad's four lanes hold the same y and all
// store it -- one address, one value -- so no per-sample branch).
template <typename TIn, int NT, bool MIX = true, int QL = 1>
__global__ __launch_bounds__(64) void k_lf_fwd(const TIn *__restrict__ x, Lay lx, int C, long M, int pad,
                                               const double *__restrict__ b, const double *__restrict__ a,
                                               const double *__restrict__ zi, const double *__restrict__ mixc,
                                               const uint8_t *__restrict__ mixon, double fs,
                                               double *__restrict__ scr, Lay ls) {
    static_assert(QL == 1 || (QL == 4 && NT == 5), "Lfilt4 holds butter(4)'s four states");
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int ch = (gid / QL) >> 1, comp = (gid / QL) & 1;
    constexpr bool st = true;
    if (ch >= C) return;   // whole quads
    const bool mix = MIX && mixon && mixon[ch];
    const double c = mix ? mixc[ch] : 0.0;
    const TIn *xp = x + lx.off(ch, 0);
    const size_t sx = lx.s_n;
    const long L = M + 2 * pad;
    typename std::conditional<QL == 4, Lfilt4, Lfilt<NT>>::type f;
    f.init(b, a, zi, lf_ext(xp, sx, M, pad, 0, comp, mix, c, fs));
    double *sp = scr + ls.off(ch, 0) + comp;
    const size_t ss = ls.s_n;
    long j = 0;
    for (; j < pad; ++j) {
        const double yv = f.step(lf_ext(xp, sx, M, pad, j, comp, mix, c, fs));
        if (st) sp[(size_t)j * ss] = yv;
    }
    // body: a batch's 16 (re, im) loads issue together, one batch ahead of the recursion; the
    // mixer (a divergent sincos branch) runs between load and recursion
    using P2 = typename std::conditional<sizeof(TIn) == 4, float2, double2>::type;
    const P2 *xq = reinterpret_cast<const P2 *>(xp);   // (re, im) of sample n at xq[n * sx / 2]
    const size_t sq = sx / 2;
    P2 ra[LFB], rb[LFB];
    auto ld = [&](P2 (&r)[LFB], long j0) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < LFB; ++u) r[u] = xq[(size_t)(j0 + u - pad) * sq];
    };
    auto run = [&](P2 (&r)[LFB], long j0) __attribute__((always_inline)) {
        double xs[LFB];
#pragma unroll
        for (int u = 0; u < LFB; ++u) xs[u] = mix_pair((double)r[u].x, (double)r[u].y, j0 + u - pad, comp, mix, c, fs);
#pragma unroll
        for (int u = 0; u < LFB; ++u) {
            const double yv = f.step(xs[u]);
            if (st) sp[(size_t)(j0 + u) * ss] = yv;
        }
    };
    if (M >= 2 * LFB) {
        ld(ra, j);
        ld(rb, j + LFB);
        for (; j + 4 * LFB <= pad + M; j += 2 * LFB) {
            run(ra, j);
            __builtin_amdgcn_sched_barrier(0);
            ld(ra, j + 2 * LFB);
            run(rb, j + LFB);
            __builtin_amdgcn_sched_barrier(0);
            ld(rb, j + 3 * LFB);
        }
        run(ra, j);
        run(rb, j + LFB);
        j += 2 * LFB;
    }
    for (; j < L; ++j) {
        const double yv = f.step(lf_ext(xp, sx, M, pad, j, comp, mix, c, fs));
        if (st) sp[(size_t)j * ss] = yv;
    }
}

// Reverse pass: y[t] = output at ext index t + pad, t in [0, M).
template <int NT, int QL = 1>
__global__ __launch_bounds__(64) void k_lf_bwd(const double *__restrict__ scr, Lay ls, int C, long M, int pad,
                                               const double *__restrict__ b, const double *__restrict__ a,
                                               const double *__restrict__ zi, double *__restrict__ out, Lay lo) {
    static_assert(QL == 1 || (QL == 4 && NT == 5), "Lfilt4 holds butter(4)'s four states");
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int ch = (gid / QL) >> 1, comp = (gid / QL) & 1;
    constexpr bool st = true;
    if (ch >= C) return;   // whole quads
    const double *sp = scr + ls.off(ch, 0) + comp;
    const size_t ss = ls.s_n;
    const long L = M + 2 * pad;
    typename std::conditional<QL == 4, Lfilt4, Lfilt<NT>>::type f;
    f.init(b, a, zi, sp[(size_t)(L - 1) * ss]);
    double *op = out + lo.off(ch, 0) + comp;
    const size_t so = lo.s_n;
    long j = L - 1;
    for (; j >= pad + M; --j) f.step(sp[(size_t)j * ss]);   // end padding: no output
    double xa[LFB], xb[LFB];
    auto ld = [&](double (&v)[LFB], long j0) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < LFB; ++u) v[u] = sp[(size_t)(j0 - u) * ss];
    };
    auto run = [&](double (&v)[LFB], long j0) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < LFB; ++u) {
            const double yv = f.step(v[u]);
            if (st) op[(size_t)(j0 - u - pad) * so] = yv;
        }
    };
    if (j - 2 * LFB + 1 >= pad) {
        ld(xa, j);
        ld(xb, j - LFB);
        for (; j - 4 * LFB + 1 >= pad; j -= 2 * LFB) {
            run(xa, j);
            __builtin_amdgcn_sched_barrier(0);
            ld(xa, j - 2 * LFB);
            run(xb, j - LFB);
            __builtin_amdgcn_sched_barrier(0);
            ld(xb, j - 3 * LFB);
        }
        run(xa, j);
        run(xb, j - LFB);
        j -= 2 * LFB;
    }
    for (; j >= 0; --j) {
        const double yn = f.step(sp[(size_t)j * ss]);
        if (st && j >= pad) op[(size_t)(j - pad) * so] = yn;
    }
}

// ------------------------------------------------------------------ time-blocked filtfilt (latency mode)
// filter_signal's lfilter passes for a few channels, parallel in time like the decimator above: one
// lane per (channel, component, tile of LB_B samples), the tile's input -- the odd extension of the
// (mixed) decimated samples, each mixed in parallel as it is loaded -- staged in LDS; pass 1 from zero
// state gives each tile's end state (the 4 DF-II-T states), k_lfb_scan the true start states in
// float64 (Psi = B^LB_B, B the one-sample zero-input transition of scipy's lfilter loop), pass 2
// the outputs.  Everything is float64, so the outputs differ from scipy's sequential pass by float64
// rounding only (oracle/compat.py: filtfilt_blocked restates it; the GPU equals it bit for bit).
constexpr int LB_B = 128;        // samples per tile
constexpr int LB_ST = 16;        // stream-tiles per workgroup (one lane of wave 0 each): one channel's
                                 // tiles spread over many CUs, 8 staged samples (and mixers) per thread
constexpr int LB_T = 256;        // threads per workgroup: all four waves stage the tiles
constexpr int LB_NS = 4;         // states (butter(4): 5 taps)

struct LbGeo {
    int C, Tn, pad;
    long M, L;
};

// stream-tile g = (ch * Tn + tile) * 2 + comp
template <typename TIn, bool FWD, bool FINAL>
__global__ __launch_bounds__(LB_T) void k_lfb_tile(const TIn *__restrict__ x, Lay lx, const double *__restrict__ mixc,
                                                    const uint8_t *__restrict__ mixon, double fs,
                                                    double *__restrict__ scr, Lay ls, LbGeo G,
                                                    const double *__restrict__ b, const double *__restrict__ a,
                                                    const double *__restrict__ states, double *__restrict__ ends,
                                                    double *__restrict__ out, Lay lo) {
    __shared__ double buf[LB_ST][LB_B + 1];
    __shared__ int rch[LB_ST], rtile[LB_ST];   // the rows' channel and tile (one division per row)
    const int tid = threadIdx.x;
    const long ntiles = (long)2 * G.C * G.Tn;
    const int nrow = (int)min((long)LB_ST, ntiles - (long)blockIdx.x * LB_ST);
    if (tid < LB_ST) {
        const int pr = (int)((((long)blockIdx.x * LB_ST + (tid < nrow ? tid : 0))) >> 1);
        rtile[tid] = pr % G.Tn;
        rch[tid] = pr / G.Tn;
    }
    __syncthreads();
    // cooperative load by all LB_T threads, 8 loads in flight per thread (unconditional, clamped),
    // then each element's value: lf_ext's arithmetic (mixer, odd extension) on the loaded samples
    constexpr int PER = LB_ST * LB_B / LB_T, U = 8;
    using P2 = typename std::conditional<sizeof(TIn) == 4, float2, double2>::type;
    auto where = [&](int i, int &r, int &j, long &e, int &ch, int &comp, bool &in) {
        r = i / LB_B;
        j = i % LB_B;
        in = r < nrow;
        const int rr = in ? r : 0;
        comp = rr & 1;   // LB_ST is even
        const int tile = rtile[rr];
        ch = rch[rr];
        e = (long)tile * LB_B + j;
        in = in && e < G.L;
        if (!in) e = 0;
    };
    for (int c0 = 0; c0 < PER; c0 += U) {
        P2 raw[U];      // forward: the input pair
        double rb[U];   // backward: the scratch value
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int r, j, ch, comp;
            long e;
            bool in;
            where(tid + LB_T * (c0 + u), r, j, e, ch, comp, in);
            if (FWD) {   // the (re, im) pair of the sample lf_ext reflects (or copies) at ext index e
                const long n = e < G.pad ? G.pad - e : (e < G.pad + G.M ? e - G.pad : G.M - 2 - (e - G.pad - G.M));
                raw[u] = *reinterpret_cast<const P2 *>(x + lx.off(ch, 0) + (size_t)n * lx.s_n);
            } else {
                rb[u] = scr[ls.off(ch, G.L - 1 - e) + comp];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int r, j, ch, comp;
            long e;
            bool in;
            where(tid + LB_T * (c0 + u), r, j, e, ch, comp, in);
            double v = 0.0;
            if (in) {
                if (FWD) {
                    const bool mix = mixon && mixon[ch];
                    const int side = e < G.pad ? -1 : (e < G.pad + G.M ? 0 : 1);
                    const long n = side < 0 ? G.pad - e : (side == 0 ? e - G.pad : G.M - 2 - (e - G.pad - G.M));
                    if (mix) {   // mixed_val on the loaded pair, then the extension in double
                        const double c = mixc[ch];
                        const double th = c * ((double)n / fs);
                        double sn, co;
                        sincos(th, &sn, &co);
                        const double xr = (double)raw[u].x, xi = (double)raw[u].y;
                        v = comp ? fma(xr, sn, xi * co) : fma(xr, co, -(xi * sn));
                        if (side != 0)
                            v = 2.0 * mixed_val(x + lx.off(ch, 0), lx.s_n, side < 0 ? 0 : G.M - 1, comp, true, c, fs) - v;
                    } else {     // the extension in the input precision, then promoted
                        const TIn vv = comp ? raw[u].y : raw[u].x;
                        if (side == 0) {
                            v = (double)vv;
                        } else {
                            const TIn ev = x[lx.off(ch, side < 0 ? 0 : G.M - 1) + comp];
                            v = (double)((TIn)2 * ev - vv);
                        }
                    }
                } else {
                    v = rb[u];
                }
            }
            buf[r][j] = v;
        }
    }
    __syncthreads();
    // the recursion: one lane of wave 0 per stream-tile
    const int row = tid < LB_ST ? tid : 0;
    const long g = (long)blockIdx.x * LB_ST + row;
    const bool own = tid < LB_ST && g < ntiles;
    const int tile = own ? (int)((g >> 1) % G.Tn) : 0;
    const int len = own ? (int)min((long)LB_B, G.L - (long)tile * LB_B) : 0;
    Lfilt<LB_NS + 1> f;
#pragma unroll
    for (int k = 0; k <= LB_NS; ++k) { f.bb[k] = b[k]; f.aa[k] = a[k]; }
#pragma unroll
    for (int k = 0; k < LB_NS; ++k) f.z[k] = (FINAL && own) ? states[g * LB_NS + k] : 0.0;
    // every tile runs all LB_B steps: the last tile of a stream (len < LB_B) steps on the zeros past
    // its end -- its end state is not used by the scan and its outputs past len are not stored
    (void)len;
    for (int j0 = 0; j0 < (tid < LB_ST ? LB_B : 0); j0 += 16) {   // wave 0 only (wave-uniform)
        double in[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) in[u] = buf[row][j0 + u];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const double y = f.step(in[u]);
            if (FINAL) buf[row][j0 + u] = y;
        }
    }
    if (!FINAL) {
        if (own) {
#pragma unroll
            for (int k = 0; k < LB_NS; ++k) ends[g * LB_NS + k] = f.z[k];
        }
        return;
    }
    __syncthreads();
    for (int i = tid; i < LB_ST * LB_B; i += LB_T) {
        const int r = i / LB_B, j = i % LB_B;
        if (r >= nrow) continue;
        const int comp = r & 1, tl = rtile[r], ch = rch[r];
        const long e = (long)tl * LB_B + j;
        if (e >= G.L) continue;
        if (FWD) {
            scr[ls.off(ch, e) + comp] = buf[r][j];
        } else {   // ext index L-1-e -> output t = ext - pad
            const long t = G.L - 1 - e - G.pad;
            if (t >= 0 && t < G.M) out[lo.off(ch, t) + comp] = buf[r][j];
        }
    }
}

// Start states of every tile of one stream (workgroup = stream 2 ch + comp, thread = tile), as
// k_sosb_scan: w_0 = zi * ext[0] (forward) or zi * scr[L-1] (backward), w_k = e_{k-1};
// w_k += Psi^d w_{k-d} for d = 1, 2, 4, .., products summed in j order without FMA.
template <typename TIn, bool FWD>
__global__ __launch_bounds__(1024) void k_lfb_scan(const TIn *__restrict__ x, Lay lx, const double *__restrict__ mixc,
                                                   const uint8_t *__restrict__ mixon, double fs,
                                                   const double *__restrict__ scr, Lay ls, LbGeo G,
                                                   const double *__restrict__ zi, const double *__restrict__ psi,
                                                   const double *__restrict__ ends, double *__restrict__ states) {
    __shared__ double w[SB_MAXT][LB_NS];
    const int k = threadIdx.x, s = blockIdx.x, ch = s >> 1, comp = s & 1;
    const bool on = k < G.Tn;
    double v[LB_NS];
    if (on) {
        if (k == 0) {
            double x0;
            if (FWD) {
                const bool mix = mixon && mixon[ch];
                x0 = lf_ext(x + lx.off(ch, 0), lx.s_n, G.M, G.pad, 0, comp, mix, mix ? mixc[ch] : 0.0, fs);
            } else {
                x0 = scr[ls.off(ch, G.L - 1) + comp];
            }
#pragma unroll
            for (int i = 0; i < LB_NS; ++i) v[i] = zi[i] * x0;
        } else {
            const double *e = ends + ((size_t)(ch * G.Tn + k - 1) * 2 + comp) * LB_NS;
#pragma unroll
            for (int i = 0; i < LB_NS; ++i) v[i] = e[i];
        }
#pragma unroll
        for (int i = 0; i < LB_NS; ++i) w[k][i] = v[i];
    }
    for (int r = 0; (1 << r) < G.Tn; ++r) {
        const int d = 1 << r;
        __syncthreads();
        double u[LB_NS];
        const bool upd = on && k >= d;
        if (upd) {
#pragma unroll
            for (int i = 0; i < LB_NS; ++i) u[i] = w[k - d][i];
        }
        __syncthreads();
        if (upd) {
            const double *P = psi + (size_t)r * LB_NS * LB_NS;
#pragma unroll
            for (int i = 0; i < LB_NS; ++i) {
                double acc = v[i];
#pragma unroll
                for (int j = 0; j < LB_NS; ++j) acc = acc + P[i * LB_NS + j] * u[j];
                v[i] = acc;
                w[k][i] = acc;
            }
        }
    }
    if (on) {
        double *o = states + ((size_t)(ch * G.Tn + k) * 2 + comp) * LB_NS;
#pragma unroll
        for (int i = 0; i < LB_NS; ++i) o[i] = v[i];
    }
}

// B (scipy lfilter's one-sample zero-input transition of the 4 DF-II-T states) and the table
// Psi^(2^r) = B^(LB_B 2^r), r < SB_NPOW, row-major 4 x 4 each; products summed in k order, no FMA.
void lfilter_table(const double *bcoef, const double *acoef, double *tab /*[SB_NPOW * 16]*/) {
    constexpr int K = LB_NS;
    double Bm[K * K];
    for (int c = 0; c < K; ++c) {
        double z[K] = {0}, zn[K];
        z[c] = 1.0;
        const double xn = 0.0;
        const double yn = z[0] + bcoef[0] * xn;
        for (int k = 0; k < K - 1; ++k) zn[k] = (z[k + 1] + xn * bcoef[k + 1]) - yn * acoef[k + 1];
        zn[K - 1] = xn * bcoef[K] - yn * acoef[K];
        for (int i = 0; i < K; ++i) Bm[i * K + c] = zn[i];
    }
    auto square = [](const double *P, double *outp) {
        double t[K * K];
        for (int i = 0; i < K; ++i)
            for (int j = 0; j < K; ++j) {
                double acc = 0.0;
                for (int k = 0; k < K; ++k) acc = acc + P[i * K + k] * P[k * K + j];
                t[i * K + j] = acc;
            }
        for (int i = 0; i < K * K; ++i) outp[i] = t[i];
    };
    for (int n = 1; n < LB_B; n <<= 1) square(Bm, Bm);
    for (int i = 0; i < K * K; ++i) tab[i] = Bm[i];
    for (int r = 1; r < SB_NPOW; ++r) square(tab + (r - 1) * K * K, tab + r * K * K);
}

// frequency_shift alone (component API, and the unfiltered-but-shifted process() path).
template <typename TIn>
__global__ __launch_bounds__(256) void k_mix(const TIn *__restrict__ x, Lay lx, int C, long N,
                                             const double *__restrict__ mixc, const uint8_t *__restrict__ mixon,
                                             double fs, double *__restrict__ out, Lay lo) {
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int ch = (int)(gid / N);
    const long n = gid - (long)ch * N;
    if (ch >= C) return;
    const bool mix = !mixon || mixon[ch];
    const TIn *xp = x + lx.off(ch, 0);
    double *op = out + lo.off(ch, n);
    op[0] = mixed_val(xp, lx.s_n, n, 0, mix, mixc[ch], fs);
    op[1] = mixed_val(xp, lx.s_n, n, 1, mix, mixc[ch], fs);
}

// The ETSI receiver's AFC mixer on a streaming window (tetra_etsi_mix): frequency_shift's
// arithmetic (mixed_val: theta = c (n / fs) in float64, sincos, numpy's complex product) with n the
// GLOBAL sample index n0 + i of the capture, rounded to cf32 -- so consecutive windows of one capture
// are mixed with one continuous phase, and the first (n0 = 0) equals the chunk mixed from its start.
__global__ __launch_bounds__(256) void k_mix_at(const float *__restrict__ x, long ld, int C, long N,
                                                const double *__restrict__ mixc, double fs, long n0,
                                                float *__restrict__ out) {
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int ch = (int)(gid / N);
    const long i = gid - (long)ch * N;
    if (ch >= C) return;
    const float *xp = x + 2 * ((size_t)ch * ld + i);
    const double xr = (double)xp[0], xi = (double)xp[1];
    const double th = mixc[ch] * ((double)(n0 + i) / fs);
    double sn, co;
    sincos(th, &sn, &co);
    out[2 * ((size_t)ch * N + i)] = (float)fma(xr, co, -(xi * sn));
    out[2 * ((size_t)ch * N + i) + 1] = (float)fma(xr, sn, xi * co);
}

// ------------------------------------------------------------------ extract_symbols
// numpy complex |z| (SIMD kernel): larger*sqrt(fma(r, r, 1)), r = smaller/larger.
template <typename T>
__device__ __forceinline__ T np_cabs(T xr, T xi) {
    T re = fabs(xr), im = fabs(xi);
    const T inf = (T)INFINITY;
    const bool re_inf = re == inf, im_inf = im == inf;
    im = re_inf ? inf : im;
    re = im_inf ? inf : re;
    const bool re_ok = !isnan(re), im_ok = !isnan(im);
    im = re_ok ? im : (T)NAN;
    re = im_ok ? re : (T)NAN;
    const T larger = fmax(re, im), smaller = fmin(im, re);
    const bool div_ok = !(larger == (T)0 || smaller == inf);
    const T r = div_ok ? smaller / larger : (T)0;
    return sqrt(fma(r, r, (T)1)) * larger;
}

// extract_symbols' element values |y[n]|^2 (numpy's |z|, squared) for every sample of every channel,
// in parallel: the latency mode's prepass, so k_extract's per-phase pairwise sums read them instead of
// each lane computing its phase's ~1000 |z| one after another.  pw rows [C][M].
template <typename T>
__global__ __launch_bounds__(256) void k_cabs2(const T *__restrict__ y, Lay ly, int C, long M, T *__restrict__ pw) {
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int ch = (int)(gid / M);
    const long n = gid - (long)ch * M;
    if (ch >= C) return;
    const size_t o = ly.off(ch, n);
    const T a = np_cabs(y[o], y[o + 1]);
    pw[(size_t)ch * M + n] = a * a;
}

// np.mean of v(0..n-1): numpy's pairwise summation (leaf blocks <= 128 with 8 accumulators,
// split point n/2 rounded down to a multiple of 8), then / n.
template <typename T, typename F>
__device__ T pairwise_mean(F v, long n) {
    long st_s[24], st_n[24];
    int st_stage[24];
    T st_left[24];
    int sp = 0;
    st_s[0] = 0; st_n[0] = n; st_stage[0] = 0; sp = 1;
    T ret = 0;
    while (sp > 0) {
        const int top = sp - 1;
        const long s = st_s[top], m = st_n[top];
        if (m <= 128) {
            if (m < 8) {
                T r = 0;
                for (long i = 0; i < m; ++i) r += v(s + i);
                ret = r;
            } else {
                T r[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) r[k] = v(s + k);
                long i = 8;
                for (; i < m - (m % 8); i += 8) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) r[k] += v(s + i + k);
                }
                T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                for (; i < m; ++i) res += v(s + i);
                ret = res;
            }
            --sp;
            continue;
        }
        long n2 = m / 2;
        n2 -= n2 % 8;
        if (st_stage[top] == 0) {
            st_stage[top] = 1;
            st_s[sp] = s; st_n[sp] = n2; st_stage[sp] = 0; ++sp;
        } else if (st_stage[top] == 1) {
            st_left[top] = ret;
            st_stage[top] = 2;
            st_s[sp] = s + n2; st_n[sp] = m - n2; st_stage[sp] = 0; ++sp;
        } else {
            ret = st_left[top] + ret;
            --sp;
        }
    }
    return ret / (T)n;
}

// The same sum as pairwise_mean's, with the tree unrolled at compile time (no stack in scratch, and
// the leaves' loads 16 deep): at most D splits, then leaves of <= 128.  A part after d splits is at
// most n / 2^d + 14 long (each split rounds down to a multiple of 8), so with D = 5 every leaf is
// <= 128 for n <= 3584; callers take pairwise_mean beyond that.  Element i is |y[ph + i sps]|^2; the
// leaf is one out-of-line function (32 inlined copies of its unrolled |z| code would be ~1 MB).
template <typename T>
struct PhasePower {
    const T *yp;
    size_t sy;
    long ph;
    int sps;
    const T *pw;   // the channel's k_cabs2 row, or null: compute |z|^2 here
    __device__ __forceinline__ T operator()(long i) const {
        if (pw) return pw[ph + i * sps];
        const size_t o = (size_t)(ph + i * sps) * sy;
        const T a = np_cabs(yp[o], yp[o + 1]);
        return a * a;
    }
};
template <typename T>
__device__ __noinline__ T pw_leaf(PhasePower<T> v, long s, long m) {
    if (m < 8) {
        T r = 0;
        for (long i = 0; i < m; ++i) r += v(s + i);
        return r;
    }
    T r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = v(s + k);
    long i = 8;
    const long mm = m - (m % 8);
    for (; i + 8 < mm; i += 16) {   // two groups of 8 loads in flight, summed in order
        T a[8], b[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            a[k] = v(s + i + k);
            b[k] = v(s + i + 8 + k);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] += a[k];
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] += b[k];
    }
    for (; i < mm; i += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] += v(s + i + k);
    }
    T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < m; ++i) res += v(s + i);
    return res;
}
template <int D, typename T>
__device__ __forceinline__ T pw_sum(const PhasePower<T> &v, long s, long n) {
    if constexpr (D == 0) {
        return pw_leaf<T>(v, s, n);   // n <= 128 here whenever the root's n <= 3584 (see above)
    } else {
        if (n <= 128) return pw_leaf<T>(v, s, n);
        long n2 = n / 2;
        n2 -= n2 % 8;
        const T l = pw_sum<D - 1, T>(v, s, n2);
        const T r = pw_sum<D - 1, T>(v, s + n2, n - n2);
        return l + r;
    }
}

// 16 lanes per channel: lane k tries phase k*step (processor.py:196-210), then the group gathers
// the chosen phase into sym[ch][0..ns).
template <typename T>
__global__ __launch_bounds__(256) void k_extract(const T *__restrict__ y, Lay ly, int C, long M, int sps, int step,
                                                 T *__restrict__ sym, long smax, int32_t *__restrict__ nsym,
                                                 int32_t *__restrict__ bestph, const T *__restrict__ pw = nullptr) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int ch = gid >> 4, k = gid & 15;
    const int lane = threadIdx.x & 63;
    const bool ok = ch < C;
    const int nph = (sps + step - 1) / step;
    const int ph = k * step;
    const T *yp = y + ly.off(ok ? ch : 0, 0);
    const size_t sy = ly.s_n;
    T power = (T)-2;
    long ns = (ok && k < nph) ? (M - ph) / sps : 0;
    if (ns > 0) {
        const PhasePower<T> v{yp, sy, (long)ph, sps, pw ? pw + (size_t)ch * M : nullptr};
        power = ns <= 3584 ? pw_sum<5, T>(v, 0, ns) / (T)ns : pairwise_mean<T>(v, ns);
    }
    T best = (T)-1;
    int bph = 0;
    for (int q = 0; q < nph && q < 16; ++q) {
        const T p = __shfl(power, (lane & ~15) + q, 64);
        const long nq = (M - q * step) / sps;
        if (nq > 0 && p > best) { best = p; bph = q * step; }
    }
    if (!ok) return;
    const long nout = (M - bph) / sps;
    if (k == 0) {
        nsym[ch] = (int32_t)nout;
        if (bestph) bestph[ch] = bph;
    }
    T *op = sym + (size_t)ch * smax * 2;
    for (long i = k; i < nout; i += 16) {
        const size_t o = (size_t)(bph + i * sps) * sy;
        op[2 * i] = yp[o];
        op[2 * i + 1] = yp[o + 1];
    }
}

// Latency mode (a few channels): one 512-thread workgroup per channel, thread = (phase q < 16, leaf
// l < 32).  numpy's pairwise sum of a phase's |y|^2 (pw_sum<5>: splits at n/2 rounded down to a
// multiple of 8 until a part is <= 128, leaves of 8 accumulators) is the same tree here, with its
// <= 32 leaves summed by 32 threads at once and combined in the tree's order by one thread: the same
// adds, so the same power, the same phase and the same symbols as k_extract.  ns <= 3584 per phase
// (five splits); longer chunks take k_extract.
constexpr int XL_LEAVES = 32;
__device__ __forceinline__ int leaf_at(long n, int want, long &s, long &m) {   // DFS leaf `want` of the tree on [0, n)
    long st_s[6], st_n[6];
    int sp = 0, idx = 0;
    st_s[0] = 0;
    st_n[0] = n;
    sp = 1;
    while (sp > 0) {
        --sp;
        const long ss = st_s[sp], nn = st_n[sp];
        if (nn <= 128) {
            if (idx == want) {
                s = ss;
                m = nn;
                return 1;
            }
            ++idx;
            continue;
        }
        long n2 = nn / 2;
        n2 -= n2 % 8;
        st_s[sp] = ss + n2;   // right pushed first: the left child is visited first
        st_n[sp] = nn - n2;
        ++sp;
        st_s[sp] = ss;
        st_n[sp] = n2;
        ++sp;
    }
    return 0;
}
template <int D, typename T>
__device__ T leaf_combine(const T *leaf, int &idx, long n) {   // pw_sum<D>'s adds over the leaf sums
    if constexpr (D == 0) {
        return leaf[idx++];
    } else {
        if (n <= 128) return leaf[idx++];
        long n2 = n / 2;
        n2 -= n2 % 8;
        const T l = leaf_combine<D - 1, T>(leaf, idx, n2);
        const T r = leaf_combine<D - 1, T>(leaf, idx, n - n2);
        return l + r;
    }
}

template <typename T>
__global__ __launch_bounds__(512) void k_extract_lat(const T *__restrict__ y, Lay ly, int C, long M, int sps, int step,
                                                     T *__restrict__ sym, long smax, int32_t *__restrict__ nsym,
                                                     int32_t *__restrict__ bestph, const T *__restrict__ pw) {
    __shared__ T leafs[16][XL_LEAVES];
    __shared__ T power[16];
    __shared__ int bsel;
    const int ch = blockIdx.x, t = threadIdx.x, q = t >> 5, l = t & 31;
    const int nph = (sps + step - 1) / step;
    const int ph = q * step;
    const long ns = q < nph ? (M - ph) / sps : 0;
    const T *yp = y + ly.off(ch, 0);
    if (ns > 0) {
        long s0, m0;
        if (leaf_at(ns, l, s0, m0)) {
            const PhasePower<T> v{yp, ly.s_n, (long)ph, sps, pw + (size_t)ch * M};
            leafs[q][l] = pw_leaf<T>(v, s0, m0);
        }
    }
    __syncthreads();
    if (l == 0) {
        T p = (T)-2;
        if (ns > 0) {
            int idx = 0;
            p = leaf_combine<5, T>(leafs[q], idx, ns) / (T)ns;
        }
        if (q < 16) power[q] = p;
    }
    __syncthreads();
    if (t == 0) {   // k_extract's choice: the first phase of the largest power
        T best = (T)-1;
        int bph = 0;
        for (int qq = 0; qq < nph && qq < 16; ++qq) {
            const long nq = (M - qq * step) / sps;
            if (nq > 0 && power[qq] > best) {
                best = power[qq];
                bph = qq * step;
            }
        }
        bsel = bph;
        nsym[ch] = (int32_t)((M - bph) / sps);
        if (bestph) bestph[ch] = bph;
    }
    __syncthreads();
    const int bph = bsel;
    const long nout = (M - bph) / sps;
    T *op = sym + (size_t)ch * smax * 2;
    for (long i = t; i < nout; i += 512) {
        const size_t o = (size_t)(bph + i * sps) * ly.s_n;
        op[2 * i] = yp[o];
        op[2 * i + 1] = yp[o + 1];
    }
}

// ------------------------------------------------------------------ demodulate_dqpsk
// sym rows [C][stride] complex T, S = nsym[ch] (or S_all); REAL: rows of real T (the reference
// called on a real array: numpy's real division and product, np.imag(diff) = +0).
// BS threads per channel: 64 for batches (one wave per channel), 1024 in the latency mode (a few
// channels: ~1 symbol per thread).  The max is order-independent, so the result is the same.
template <typename T, int BS, bool REAL = false>
__global__ __launch_bounds__(BS) void k_demod(const T *__restrict__ sym, long stride, int C, const int32_t *__restrict__ nsym,
                                              long S_all, double t0, double t1, double t2, double t3,
                                              uint8_t *__restrict__ hard, long hstride) {
    const int ch = blockIdx.x;
    const int lane = threadIdx.x;
    if (ch >= C) return;
    const long S = nsym ? nsym[ch] : S_all;
    if (S < 2) return;
    const T *sp = sym + (size_t)ch * stride * (REAL ? 1 : 2);
    T m = (T)-INFINITY;
    bool any_nan = false;
    for (long k = lane; k < S; k += BS) {
        const T a = REAL ? fabs(sp[k]) : np_cabs(sp[2 * k], sp[2 * k + 1]);
        any_nan |= isnan(a);
        m = fmax(m, a);
    }
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    any_nan = __any(any_nan);
    if constexpr (BS > 64) {   // across the waves
        __shared__ T wm[BS / 64];
        __shared__ int wn[BS / 64];
        if ((lane & 63) == 0) {
            wm[lane >> 6] = m;
            wn[lane >> 6] = any_nan;
        }
        __syncthreads();
        m = wm[0];
        any_nan = wn[0];
        for (int w = 1; w < BS / 64; ++w) {
            m = fmax(m, wm[w]);
            any_nan |= wn[w] != 0;
        }
    }
    const T mx = any_nan ? (T)NAN : m;   // np.max propagates NaN
    // samples / max_power: numpy complex division (Smith) by (m + 0j): rat = 0/m, scl = 1/m,
    // out = ((xr + xi*rat)*scl, (xi - xr*rat)*scl)
    const bool norm = mx > (T)0;
    const T rat = norm ? (T)0 / mx : (T)0;
    const T scl = norm ? (T)1 / (mx + (T)0 * rat) : (T)1;
    const T th0 = (T)t0, th1 = (T)t1, th2 = (T)t2, th3 = (T)t3;
    uint8_t *hp = hard + (size_t)ch * hstride;
    if constexpr (REAL) {
        // samples / max_power then sample * conj(prev) on real scalars: the product's sign (and
        // signed zero) decides; arctan2(+0, dr) is 0 or pi
        for (long k = 1 + lane; k < S; k += BS) {
            T sr = sp[k], pr = sp[k - 1];
            if (norm) {
                sr = sr / mx;
                pr = pr / mx;
            }
            const T ph = atan2((T)0, sr * pr);
            hp[k - 1] = ph < th0 ? 3 : ph < th1 ? 2 : ph < th2 ? 0 : ph < th3 ? 1 : 3;
        }
        return;
    }
    for (long k = 1 + lane; k < S; k += BS) {
        T sr = sp[2 * k], si = sp[2 * k + 1], pr = sp[2 * k - 2], pi = sp[2 * k - 1];
        if (norm) {
            const T a = (sr + si * rat) * scl, b = (si - sr * rat) * scl;
            const T c = (pr + pi * rat) * scl, d = (pi - pr * rat) * scl;
            sr = a; si = b; pr = c; pi = d;
        }
        // numpy scalar complex multiply sample * conj(prev), no FMA
        const T npi = -pi;
        const T dr = sr * pr - si * npi;
        const T di = sr * npi + si * pr;
        const T ph = atan2(di, dr);
        uint8_t s;
        if (ph < th0) s = 3;
        else if (ph < th1) s = 2;
        else if (ph < th2) s = 0;
        else if (ph < th3) s = 1;
        else s = 3;
        hp[k - 1] = s;
    }
}

// grouped [C/32][len][32][2] -> row-major [C][len] complex
template <typename T>
__global__ void k_relayout(const T *__restrict__ in, Lay li, int C, long len, T *__restrict__ out, Lay lo) {
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int ch = (int)(gid / len);
    const long n = gid - (long)ch * len;
    if (ch >= C) return;
    const T *ip = in + li.off(ch, n);
    T *op = out + lo.off(ch, n);
    op[0] = ip[0];
    op[1] = ip[1];
}

long ceil_div(long a, long b) { return (a + b - 1) / b; }

// ----------------------------------------------------------------- host-side stage drivers
template <typename T>
int run_decimate(tetra_ctx *ctx, const tetra_compat_plan *P, const T *x, Lay lx, int C, long N, T *out, Lay lo) {
    (void)lx;   // input rows are complex [C][N] (row_major)
    const int pad = 27;   // 3 * (2*4 + 1): sosfiltfilt default padlen for 4 sections
    const long L = N + 2 * pad;
    const long Lp = (L + 3) & ~3L;   // stream-major scratch rows, 16-byte aligned
    T *scr = (T *)ws(ctx, S_W0, (size_t)2 * C * Lp * sizeof(T));
    T *coef = (T *)ws(ctx, S_W7, 32 * sizeof(T));
    if (!scr || !coef) return TETRA_E_NOMEM;
    T hc[32];
    for (int i = 0; i < 24; ++i) hc[i] = std::is_same<T, float>::value ? (T)P->sos_f32[i] : (T)P->sos_f64[i];
    for (int i = 0; i < 8; ++i) hc[24 + i] = std::is_same<T, float>::value ? (T)P->zi_f32[i] : (T)P->zi_f64[i];
    HIP_TRY(ctx, hipMemcpyAsync(coef, hc, sizeof hc, hipMemcpyHostToDevice, ctx->stream));
    // four waves per workgroup: one per SIMD of a CU.  The 8 C lanes make one wave per SIMD over the
    // chip, and 64-lane workgroups left the placement to the dispatcher
    const unsigned blk = 256;
    const dim3 grid(grid_for((size_t)8 * C, blk));
    {
        PROF(ctx, "compat_sos_fwd");
        bool two = false;
        if constexpr (std::is_same<T, float>::value) {
            two = true;   // complex64: banked lanes, unique loads (any row length)
            hipLaunchKernelGGL(k_sos_fwd_bank, grid, dim3(blk), 0, ctx->stream, x, C, N, pad, coef, coef + 24, scr,
                               Lp);
        }
        if (!two)
            hipLaunchKernelGGL((k_sos_fwd<T, 1>), grid, dim3(blk), 0, ctx->stream, x, C, N, pad, coef, coef + 24, scr,
                               Lp);
    }
    {
        PROF(ctx, "compat_sos_bwd");
        // the decimation factors of 2.4 and 1.8 MSps captures (q = 10, 7) compiled in; others generic
        bool bank = false;
        if constexpr (std::is_same<T, float>::value) {
            bank = true;
            if (P->q == 10)
                hipLaunchKernelGGL((k_sos_bwd_bank<10>), grid, dim3(blk), 0, ctx->stream, scr, Lp, C, N, pad, P->q,
                                   coef, coef + 24, out, lo);
            else if (P->q == 7)
                hipLaunchKernelGGL((k_sos_bwd_bank<7>), grid, dim3(blk), 0, ctx->stream, scr, Lp, C, N, pad, P->q,
                                   coef, coef + 24, out, lo);
            else
                bank = false;
        }
        if (bank) {
        } else if (P->q == 10)
            hipLaunchKernelGGL((k_sos_bwd<T, 10>), grid, dim3(blk), 0, ctx->stream, scr, Lp, C, N, pad, P->q, coef,
                               coef + 24, out, lo);
        else if (P->q == 7)
            hipLaunchKernelGGL((k_sos_bwd<T, 7>), grid, dim3(blk), 0, ctx->stream, scr, Lp, C, N, pad, P->q, coef,
                               coef + 24, out, lo);
        else
            hipLaunchKernelGGL((k_sos_bwd<T, 0>), grid, dim3(blk), 0, ctx->stream, scr, Lp, C, N, pad, P->q, coef,
                               coef + 24, out, lo);
    }
    return TETRA_OK;
}

// The time-blocked decimator (k_sosb_*): same contract as run_decimate (complex rows [C][N] in,
// decimate's output to `out` in layout lo), with the tile geometry checked by blocked_fits.
bool blocked_fits(int C, long N, int q) {
    return C >= 1 && C <= SB_MAXC && q >= 2 && q <= SB_MAXQ && N > 27 && (N + 54 + SB_B - 1) / SB_B <= SB_MAXT;
}

template <typename T>
int run_decimate_blocked(tetra_ctx *ctx, const tetra_compat_plan *P, const T *x, int C, long N, T *out, Lay lo) {
    const int pad = 27;
    const long L = N + 2 * pad;
    const long Lp = (L + 3) & ~3L;
    const int Tn = (int)ceil_div(L, SB_B);
    const size_t ntile = (size_t)2 * C * Tn;
    T *scr = (T *)ws(ctx, S_W0, (size_t)2 * C * Lp * sizeof(T));
    T *coef = (T *)ws(ctx, S_W7, 32 * sizeof(T));
    double *sb = (double *)ws(ctx, S_W16, (2 * ntile * 8 + SB_NPOW * 64) * sizeof(double));
    if (!scr || !coef || !sb) return TETRA_E_NOMEM;
    double *ends = sb, *states = sb + ntile * 8, *phi = sb + 2 * ntile * 8;
    T hc[32];
    double dc[24];
    for (int i = 0; i < 24; ++i) {
        hc[i] = std::is_same<T, float>::value ? (T)P->sos_f32[i] : (T)P->sos_f64[i];
        dc[i] = (double)hc[i];
    }
    for (int i = 0; i < 8; ++i) hc[24 + i] = std::is_same<T, float>::value ? (T)P->zi_f32[i] : (T)P->zi_f64[i];
    // the table is a function of the 24 SOS coefficients alone (in the working precision): key the
    // upload on them, not on q, so a caller's own plan with other coefficients never reuses it
    if (!ctx->sosb_valid || ctx->sosb_dev != (const void *)phi || std::memcmp(ctx->sosb_coef, dc, sizeof dc) != 0) {
        ctx->sosb_tab.resize(SB_NPOW * 64);
        blocked_table(dc, ctx->sosb_tab.data());
        HIP_TRY(ctx, hipMemcpyAsync(phi, ctx->sosb_tab.data(), SB_NPOW * 64 * sizeof(double), hipMemcpyHostToDevice,
                                    ctx->stream));
        std::memcpy(ctx->sosb_coef, dc, sizeof dc);
        ctx->sosb_valid = true;
        ctx->sosb_dev = phi;
    }
    HIP_TRY(ctx, hipMemcpyAsync(coef, hc, sizeof hc, hipMemcpyHostToDevice, ctx->stream));
    const SbGeo G{C, Tn, pad, P->q, N, L, Lp};
    constexpr int ST = SbCfg<T>::ST;
    const dim3 gt((unsigned)ceil_div((long)ntile, ST)), bt(SB_LT);
    const dim3 gs((unsigned)(2 * C)), bs((unsigned)std::min(SB_MAXT, (int)ceil_div(Tn, 64) * 64));
    {
        PROF(ctx, "compat_sosb_fwd");
        hipLaunchKernelGGL((k_sosb_tile<T, true, false>), gt, bt, 0, ctx->stream, x, scr, G, coef, nullptr, ends,
                           (T *)nullptr, lo);
        hipLaunchKernelGGL((k_sosb_scan<T, true>), gs, bs, 0, ctx->stream, x, scr, G, coef + 24, phi, ends, states);
        hipLaunchKernelGGL((k_sosb_tile<T, true, true>), gt, bt, 0, ctx->stream, x, scr, G, coef, states, nullptr,
                           (T *)nullptr, lo);
    }
    {
        PROF(ctx, "compat_sosb_bwd");
        hipLaunchKernelGGL((k_sosb_tile<T, false, false>), gt, bt, 0, ctx->stream, x, scr, G, coef, nullptr, ends,
                           (T *)nullptr, lo);
        hipLaunchKernelGGL((k_sosb_scan<T, false>), gs, bs, 0, ctx->stream, x, scr, G, coef + 24, phi, ends, states);
        hipLaunchKernelGGL((k_sosb_tile<T, false, true>), gt, bt, 0, ctx->stream, x, scr, G, coef, states, nullptr, out,
                           lo);
    }
    HIP_TRY(ctx, hipGetLastError());
    return TETRA_OK;
}

template <typename TIn>
int run_filtfilt(tetra_ctx *ctx, const tetra_compat_plan *P, const TIn *x, Lay lx, int C, long M,
                 const double *mixc, const uint8_t *mixon, double *out, Lay lo) {
    const int nt = P->ntaps, pad = 3 * nt;
    if (nt != 5) return tetra_fail(ctx, TETRA_E_INVALID, "ntaps %d unsupported (butter(4) has 5)", nt);
    const long L = M + 2 * pad;
    double *scr = (double *)ws(ctx, S_W2, grouped_elems(C, L) * sizeof(double));
    double *coef = (double *)ws(ctx, S_W6, 3 * MAXTAP * sizeof(double));
    if (!scr || !coef) return TETRA_E_NOMEM;
    double hc[3 * MAXTAP] = {0};
    for (int k = 0; k < nt; ++k) { hc[k] = P->b[k]; hc[MAXTAP + k] = P->a[k]; }
    for (int k = 0; k < nt - 1; ++k) hc[2 * MAXTAP + k] = P->lzi[k];
    HIP_TRY(ctx, hipMemcpyAsync(coef, hc, sizeof hc, hipMemcpyHostToDevice, ctx->stream));
    const unsigned blk = 64;
    const int ql = lf_lanes(C);
    {
        PROF(ctx, "compat_filtfilt_fwd");
        const dim3 g1(grid_for((size_t)2 * C, blk)), g4(grid_for((size_t)8 * C, blk));
        const Lay ls = grouped(L);
        const double *cb = coef, *ca = coef + MAXTAP, *cz = coef + 2 * MAXTAP;
        if (ql == 4 && mixon)
            hipLaunchKernelGGL((k_lf_fwd<TIn, 5, true, 4>), g4, dim3(blk), 0, ctx->stream, x, lx, C, M, pad, cb, ca, cz,
                               mixc, mixon, P->fs_dec, scr, ls);
        else if (ql == 4)
            hipLaunchKernelGGL((k_lf_fwd<TIn, 5, false, 4>), g4, dim3(blk), 0, ctx->stream, x, lx, C, M, pad, cb, ca, cz,
                               mixc, mixon, P->fs_dec, scr, ls);
        else if (mixon)
            hipLaunchKernelGGL((k_lf_fwd<TIn, 5>), g1, dim3(blk), 0, ctx->stream, x, lx, C, M, pad, cb, ca, cz, mixc,
                               mixon, P->fs_dec, scr, ls);
        else
            hipLaunchKernelGGL((k_lf_fwd<TIn, 5, false>), g1, dim3(blk), 0, ctx->stream, x, lx, C, M, pad, cb, ca, cz,
                               mixc, mixon, P->fs_dec, scr, ls);
    }
    {
        PROF(ctx, "compat_filtfilt_bwd");
        if (ql == 4)
            hipLaunchKernelGGL((k_lf_bwd<5, 4>), dim3(grid_for((size_t)8 * C, blk)), dim3(blk), 0, ctx->stream, scr,
                               grouped(L), C, M, pad, coef, coef + MAXTAP, coef + 2 * MAXTAP, out, lo);
        else
            hipLaunchKernelGGL(k_lf_bwd<5>, dim3(grid_for((size_t)2 * C, blk)), dim3(blk), 0, ctx->stream, scr,
                               grouped(L), C, M, pad, coef, coef + MAXTAP, coef + 2 * MAXTAP, out, lo);
    }
    return TETRA_OK;
}

bool lf_blocked_fits(int C, long M, int ntaps) {
    return C >= 1 && C <= SB_MAXC && ntaps == LB_NS + 1 && (M + 6 * ntaps + LB_B - 1) / LB_B <= SB_MAXT;
}

template <typename TIn>
int run_filtfilt_blocked(tetra_ctx *ctx, const tetra_compat_plan *P, const TIn *x, Lay lx, int C, long M,
                         const double *mixc, const uint8_t *mixon, double *out, Lay lo) {
    const int nt = P->ntaps, pad = 3 * nt;
    const long L = M + 2 * pad;
    const int Tn = (int)ceil_div(L, LB_B);
    const size_t ntile = (size_t)2 * C * Tn;
    double *scr = (double *)ws(ctx, S_W2, grouped_elems(C, L) * sizeof(double));
    double *coef = (double *)ws(ctx, S_W6, (3 * MAXTAP + SB_NPOW * LB_NS * LB_NS) * sizeof(double));
    double *lb = (double *)ws(ctx, S_W17, 2 * ntile * LB_NS * sizeof(double));
    if (!scr || !coef || !lb) return TETRA_E_NOMEM;
    double hc[3 * MAXTAP + SB_NPOW * LB_NS * LB_NS] = {0};
    for (int k = 0; k < nt; ++k) { hc[k] = P->b[k]; hc[MAXTAP + k] = P->a[k]; }
    for (int k = 0; k < nt - 1; ++k) hc[2 * MAXTAP + k] = P->lzi[k];
    lfilter_table(P->b, P->a, hc + 3 * MAXTAP);
    HIP_TRY(ctx, hipMemcpyAsync(coef, hc, sizeof hc, hipMemcpyHostToDevice, ctx->stream));
    double *ends = lb, *states = lb + ntile * LB_NS;
    const double *psi = coef + 3 * MAXTAP;
    const LbGeo G{C, Tn, pad, M, L};
    const dim3 gt((unsigned)ceil_div((long)ntile, LB_ST)), bt(LB_T);
    const dim3 gs((unsigned)(2 * C)), bs((unsigned)std::min(SB_MAXT, (int)ceil_div(Tn, 64) * 64));
    const Lay ls = grouped(L);
    {
        PROF(ctx, "compat_lfb_fwd");
        hipLaunchKernelGGL((k_lfb_tile<TIn, true, false>), gt, bt, 0, ctx->stream, x, lx, mixc, mixon, P->fs_dec, scr,
                           ls, G, coef, coef + MAXTAP, nullptr, ends, nullptr, lo);
        hipLaunchKernelGGL((k_lfb_scan<TIn, true>), gs, bs, 0, ctx->stream, x, lx, mixc, mixon, P->fs_dec, scr, ls, G,
                           coef + 2 * MAXTAP, psi, ends, states);
        hipLaunchKernelGGL((k_lfb_tile<TIn, true, true>), gt, bt, 0, ctx->stream, x, lx, mixc, mixon, P->fs_dec, scr,
                           ls, G, coef, coef + MAXTAP, states, nullptr, nullptr, lo);
    }
    {
        PROF(ctx, "compat_lfb_bwd");
        hipLaunchKernelGGL((k_lfb_tile<TIn, false, false>), gt, bt, 0, ctx->stream, x, lx, mixc, mixon, P->fs_dec, scr,
                           ls, G, coef, coef + MAXTAP, nullptr, ends, nullptr, lo);
        hipLaunchKernelGGL((k_lfb_scan<TIn, false>), gs, bs, 0, ctx->stream, x, lx, mixc, mixon, P->fs_dec, scr, ls, G,
                           coef + 2 * MAXTAP, psi, ends, states);
        hipLaunchKernelGGL((k_lfb_tile<TIn, false, true>), gt, bt, 0, ctx->stream, x, lx, mixc, mixon, P->fs_dec, scr,
                           ls, G, coef, coef + MAXTAP, states, nullptr, out, lo);
    }
    HIP_TRY(ctx, hipGetLastError());
    return TETRA_OK;
}

template <typename T>
void launch_extract(tetra_ctx *ctx, const T *y, Lay ly, int C, long M, int sps, int step, T *sym, long smax,
                    int32_t *nsym, int32_t *bph, T *pw = nullptr) {
    PROF(ctx, "compat_extract");
    if (pw)   // latency mode: every |y|^2 first, in parallel
        hipLaunchKernelGGL(k_cabs2<T>, dim3(grid_for((size_t)C * M, 256)), dim3(256), 0, ctx->stream, y, ly, C, M, pw);
    if (pw && M / sps <= 3584)   // ... and each phase's pairwise sum leaf-parallel
        hipLaunchKernelGGL(k_extract_lat<T>, dim3(C), dim3(512), 0, ctx->stream, y, ly, C, M, sps, step, sym, smax, nsym,
                           bph, (const T *)pw);
    else
        hipLaunchKernelGGL(k_extract<T>, dim3(grid_for((size_t)16 * C, 256)), dim3(256), 0, ctx->stream, y, ly, C, M, sps,
                           step, sym, smax, nsym, bph, (const T *)pw);
}

template <typename T, bool REAL = false>
void launch_demod(tetra_ctx *ctx, const T *sym, long stride, int C, const int32_t *nsym, long S_all,
                  const double *thr, uint8_t *hard, long hstride) {
    PROF(ctx, "compat_demod");
    if (C <= SB_MAXC)   // a few channels: a workgroup of 1024 per channel
        hipLaunchKernelGGL((k_demod<T, 1024, REAL>), dim3(C), dim3(1024), 0, ctx->stream, sym, stride, C, nsym, S_all,
                           thr[0], thr[1], thr[2], thr[3], hard, hstride);
    else
        hipLaunchKernelGGL((k_demod<T, 64, REAL>), dim3(C), dim3(64), 0, ctx->stream, sym, stride, C, nsym, S_all,
                           thr[0], thr[1], thr[2], thr[3], hard, hstride);
}

// Which kernels tetra_demod_compat runs for this plan and batch shape (TETRA_FORM_* bits).
// The default (flags 0 or TETRA_COMPAT_SEQUENTIAL) is scipy's sequential operation order in both
// recursions -- bit-identical to the reference; the time-blocked forms only under
// TETRA_COMPAT_BLOCKED (the blocked decimator drifts up to 1.45e-5 from scipy's fp32
// state and can flip decisions whose margin is ~1e-6 rad, so it must be asked for).
unsigned compat_forms(const tetra_compat_plan *P, size_t C, size_t N) {
    unsigned f = 0;
    const long M = P->q > 1 ? ceil_div((long)N, P->q) : (long)N;
    if (P->flags & TETRA_COMPAT_BLOCKED) {
        if (P->q > 1 && blocked_fits((int)std::min<size_t>(C, 1 << 30), (long)N, P->q)) f |= TETRA_FORM_DEC_BLOCKED;
        if (P->filt && lf_blocked_fits((int)std::min<size_t>(C, 1 << 30), M, P->ntaps)) f |= TETRA_FORM_LF_BLOCKED;
    }
    if (C >= 1 && C <= SB_MAXC) f |= TETRA_FORM_POW_PREPASS;
    return f;
}

int check_plan(tetra_ctx *ctx, const tetra_compat_plan *P) {
    if (!P) return tetra_fail(ctx, TETRA_E_INVALID, "plan is NULL");
    if (P->sps < 1 || P->phase_step < 1) return tetra_fail(ctx, TETRA_E_INVALID, "bad sps/phase_step");
    return TETRA_OK;
}

}  // namespace

extern "C" {

int tetra_compat_forms(const tetra_compat_plan *P, size_t C, size_t N, int32_t *forms) {
    if (!P || !forms) return TETRA_E_INVALID;
    *forms = (int32_t)compat_forms(P, C, N);
    return TETRA_OK;
}

int tetra_compat_blocked_table(const tetra_compat_plan *P, int which, double *table) {
    if (!P || !table || which < 0 || which > 2) return TETRA_E_INVALID;
    if (which == 2) {   // filtfilt's lfilter
        if (P->ntaps != LB_NS + 1) return TETRA_E_INVALID;
        lfilter_table(P->b, P->a, table);
        return TETRA_OK;
    }
    double dc[24];
    for (int i = 0; i < 24; ++i) dc[i] = which ? P->sos_f64[i] : (double)P->sos_f32[i];
    blocked_table(dc, table);
    return TETRA_OK;
}

int64_t tetra_compat_symbols(const tetra_compat_plan *P, size_t N) {
    if (!P || N == 0) return 0;
    long M = P->q > 1 ? ceil_div((long)N, P->q) : (long)N;
    return M / (P->sps < 1 ? 1 : P->sps) + 1;   // upper bound over phases
}

int tetra_decimate(tetra_ctx *ctx, const tetra_compat_plan *P, const void *iq, int fmt, size_t C, size_t N, void *out) {
    if (!ctx) return TETRA_E_INVALID;
    int rc = check_plan(ctx, P);
    if (rc) return rc;
    if (P->q < 2 || N <= 27 || C == 0) return tetra_fail(ctx, TETRA_E_INVALID, "decimate needs q>=2 and N>27");
    if (fmt != TETRA_CF32 && fmt != TETRA_CF64) return tetra_fail(ctx, TETRA_E_INVALID, "compat path takes cf32/cf64");
    const size_t es = fmt == TETRA_CF64 ? 8 : 4;
    const long M = ceil_div((long)N, P->q);
    Staging st(ctx);
    const void *x = st.in(iq, C * N * 2 * es);
    void *o = st.out(out, C * M * 2 * es);
    if (!x || !o) return st.finish();
    if (fmt == TETRA_CF64)
        rc = run_decimate<double>(ctx, P, (const double *)x, row_major(N), (int)C, (long)N, (double *)o, row_major(M));
    else
        rc = run_decimate<float>(ctx, P, (const float *)x, row_major(N), (int)C, (long)N, (float *)o, row_major(M));
    if (rc) return rc;
    return st.finish();
}

int tetra_frequency_shift(tetra_ctx *ctx, const void *iq, int fmt, size_t C, size_t N, const double *mix_c, double fs,
                          void *out) {
    if (!ctx || C == 0) return TETRA_E_INVALID;
    if (N == 0) return TETRA_OK;
    if (fmt != TETRA_CF32 && fmt != TETRA_CF64) return tetra_fail(ctx, TETRA_E_INVALID, "compat path takes cf32/cf64");
    const size_t es = fmt == TETRA_CF64 ? 8 : 4;
    Staging st(ctx);
    const void *x = st.in(iq, C * N * 2 * es);
    const double *mc = (const double *)st.in(mix_c, C * sizeof(double));
    void *o = st.out(out, C * N * 16);
    if (!x || !mc || !o) return st.finish();
    const unsigned blk = 256;
    if (fmt == TETRA_CF64)
        hipLaunchKernelGGL(k_mix<double>, dim3(grid_for(C * N, blk)), dim3(blk), 0, ctx->stream, (const double *)x,
                           row_major(N), (int)C, (long)N, mc, (const uint8_t *)nullptr, fs, (double *)o, row_major(N));
    else
        hipLaunchKernelGGL(k_mix<float>, dim3(grid_for(C * N, blk)), dim3(blk), 0, ctx->stream, (const float *)x,
                           row_major(N), (int)C, (long)N, mc, (const uint8_t *)nullptr, fs, (double *)o, row_major(N));
    return st.finish();
}

int tetra_etsi_mix(tetra_ctx *ctx, const void *iq, size_t C, size_t ld, size_t N, const double *mix_c, double fs,
                   int64_t n0, void *out) {
    if (!ctx || C == 0 || ld < N) return TETRA_E_INVALID;
    if (N == 0) return TETRA_OK;
    Staging st(ctx);
    const float *x = (const float *)st.in(iq, ((C - 1) * ld + N) * 8);
    const double *mc = (const double *)st.in(mix_c, C * sizeof(double));
    float *o = (float *)st.out(out, C * N * 8);
    if (!x || !mc || !o) return st.finish();
    hipLaunchKernelGGL(k_mix_at, dim3(grid_for(C * N, 256)), dim3(256), 0, ctx->stream, x, (long)ld, (int)C, (long)N,
                       mc, fs, (long)n0, o);
    return st.finish();
}

int tetra_filtfilt(tetra_ctx *ctx, const tetra_compat_plan *P, const void *iq, int fmt, size_t C, size_t N, void *out) {
    if (!ctx) return TETRA_E_INVALID;
    if (!P || (long)N <= 3 * P->ntaps || C == 0)
        return tetra_fail(ctx, TETRA_E_INVALID, "filtfilt needs N > padlen");
    if (fmt != TETRA_CF32 && fmt != TETRA_CF64) return tetra_fail(ctx, TETRA_E_INVALID, "compat path takes cf32/cf64");
    const size_t es = fmt == TETRA_CF64 ? 8 : 4;
    Staging st(ctx);
    const void *x = st.in(iq, C * N * 2 * es);
    void *o = st.out(out, C * N * 16);
    if (!x || !o) return st.finish();
    int rc;
    if (fmt == TETRA_CF64)
        rc = run_filtfilt<double>(ctx, P, (const double *)x, row_major(N), (int)C, (long)N, nullptr, nullptr,
                                  (double *)o, row_major(N));
    else
        rc = run_filtfilt<float>(ctx, P, (const float *)x, row_major(N), (int)C, (long)N, nullptr, nullptr,
                                 (double *)o, row_major(N));
    if (rc) return rc;
    return st.finish();
}

int tetra_extract_symbols(tetra_ctx *ctx, const void *x, int fmt, size_t C, size_t N, int sps, int step, void *sym,
                          int32_t *nsym, int32_t *bestph, size_t smax) {
    if (!ctx || C == 0 || N == 0 || sps < 1 || step < 1) return tetra_fail(ctx, TETRA_E_INVALID, "bad extract args");
    if ((sps + step - 1) / step > 16) return tetra_fail(ctx, TETRA_E_INVALID, "more than 16 phases");
    if (fmt != TETRA_CF32 && fmt != TETRA_CF64) return tetra_fail(ctx, TETRA_E_INVALID, "compat path takes cf32/cf64");
    const size_t es = fmt == TETRA_CF64 ? 8 : 4;
    Staging st(ctx);
    const void *xd = st.in(x, C * N * 2 * es);
    void *sd = st.out(sym, C * smax * 2 * es);
    int32_t *nd = (int32_t *)st.out(nsym, C * 4);
    int32_t *bd = bestph ? (int32_t *)st.out(bestph, C * 4) : nullptr;
    if (!xd || !sd || !nd) return st.finish();
    if (fmt == TETRA_CF64)
        launch_extract<double>(ctx, (const double *)xd, row_major(N), (int)C, (long)N, sps, step, (double *)sd,
                               (long)smax, nd, bd);
    else
        launch_extract<float>(ctx, (const float *)xd, row_major(N), (int)C, (long)N, sps, step, (float *)sd,
                              (long)smax, nd, bd);
    return st.finish();
}

int tetra_demod_dqpsk(tetra_ctx *ctx, const void *sym, int fmt, size_t C, size_t S, const double *thr4, uint8_t *hard) {
    if (!ctx || !thr4) return TETRA_E_INVALID;
    if (S < 2 || C == 0) return TETRA_OK;
    const bool real = fmt == TETRA_F32 || fmt == TETRA_F64;
    if (fmt != TETRA_CF32 && fmt != TETRA_CF64 && !real)
        return tetra_fail(ctx, TETRA_E_INVALID, "demod_dqpsk takes cf32/cf64/f32/f64");
    const size_t es = fmt == TETRA_CF64 || fmt == TETRA_F64 ? 8 : 4;
    Staging st(ctx);
    const void *sd = st.in(sym, C * S * (real ? 1 : 2) * es);
    uint8_t *hd = (uint8_t *)st.out(hard, C * (S - 1));
    if (!sd || !hd) return st.finish();
    if (fmt == TETRA_F64)
        launch_demod<double, true>(ctx, (const double *)sd, (long)S, (int)C, nullptr, (long)S, thr4, hd, (long)(S - 1));
    else if (fmt == TETRA_F32)
        launch_demod<float, true>(ctx, (const float *)sd, (long)S, (int)C, nullptr, (long)S, thr4, hd, (long)(S - 1));
    else if (fmt == TETRA_CF64)
        launch_demod<double>(ctx, (const double *)sd, (long)S, (int)C, nullptr, (long)S, thr4, hd, (long)(S - 1));
    else
        launch_demod<float>(ctx, (const float *)sd, (long)S, (int)C, nullptr, (long)S, thr4, hd, (long)(S - 1));
    return st.finish();
}

// The sequential filtfilt takes its mixed input from a parallel k_mix pass (instead of the mixer
// inside its recursion) for batches of up to PREMIX_MAXC channels whose rows are all mixed, when the
// flags are host memory (no read-back).  Past that the batch's lanes hide the mixer's latency, and a
// float64 row written and read again would cost more than it saves (the bench's 8192 channels).
constexpr size_t PREMIX_MAXC = 64;
static bool premix_fits(size_t C, const uint8_t *mix_on) {
    if (C > PREMIX_MAXC || !mix_on || is_device_ptr(mix_on)) return false;
    for (size_t c = 0; c < C; ++c)
        if (!mix_on[c]) return false;
    return true;
}

int tetra_demod_compat(tetra_ctx *ctx, const tetra_compat_plan *P, const void *iq, int fmt, size_t C, size_t N,
                       const double *mix_c, const uint8_t *mix_on, void *soft, uint8_t *hard, int32_t *nsym,
                       size_t smax, int32_t *soft_f32) {
    if (!ctx) return TETRA_E_INVALID;
    int rc = check_plan(ctx, P);
    if (rc) return rc;
    if (C == 0 || N == 0) return tetra_fail(ctx, TETRA_E_INVALID, "empty batch (process() handles len 0 on host)");
    if ((P->sps + P->phase_step - 1) / P->phase_step > 16) return tetra_fail(ctx, TETRA_E_INVALID, "more than 16 phases");
    const bool dec = P->q > 1;
    if (dec && (int)(fmt == TETRA_CF64) != P->dec_f64) return tetra_fail(ctx, TETRA_E_INVALID, "plan/iq precision mismatch");
    const long M = dec ? ceil_div((long)N, P->q) : (long)N;
    if ((long)smax < M / P->sps + 1 && (long)smax < M) return tetra_fail(ctx, TETRA_E_INVALID, "smax too small");
    if (fmt != TETRA_CF32 && fmt != TETRA_CF64) return tetra_fail(ctx, TETRA_E_INVALID, "compat path takes cf32/cf64");
    const size_t es = fmt == TETRA_CF64 ? 8 : 4;
    Staging st(ctx);
    const void *x = st.in(iq, C * N * 2 * es);
    const double *mc = (const double *)st.in(mix_c, C * sizeof(double));
    const uint8_t *mo = (const uint8_t *)st.in(mix_on, C);
    if (!x || !mc || !mo) return st.finish();
    // mixed precision of the unfiltered path is per channel; require it uniform (host splits)
    uint8_t any_mix = 0, all_mix = 1;
    if (!P->filt) {
        std::vector<uint8_t> h(C);
        HIP_TRY(ctx, hipMemcpyAsync(h.data(), mo, C, hipMemcpyDefault, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        for (auto v : h) { any_mix |= v; all_mix &= v; }
        if (any_mix && !all_mix) return tetra_fail(ctx, TETRA_E_INVALID, "unfiltered batch with mixed freq_offset flags");
    }
    const bool f32_soft = !P->filt && !any_mix && fmt == TETRA_CF32;
    const size_t ses = f32_soft ? 4 : 8;
    void *so = st.out(soft, C * smax * 2 * ses);
    uint8_t *ho = (uint8_t *)st.out(hard, C * smax);
    int32_t *no = (int32_t *)st.out(nsym, C * 4);
    if (!so || !ho || !no) return st.finish();
    // stage 1: decimate (processor.py:248-257)
    const void *d = x;
    Lay ld = row_major(N);
    if (dec) {
        void *db = ws(ctx, S_W1, grouped_elems((int)C, M) * es);
        if (!db) return TETRA_E_NOMEM;
        // scipy's sequential operation order unless the caller opts into the latency mode
        // (TETRA_COMPAT_BLOCKED: parallel in time, within the filter's fp32 noise of scipy, not
        // bit-exact -- see compat_forms)
        const bool blocked = compat_forms(P, C, N) & TETRA_FORM_DEC_BLOCKED;
        if ((P->flags & TETRA_COMPAT_BLOCKED) && !blocked_fits((int)C, (long)N, P->q))
            return tetra_fail(ctx, TETRA_E_INVALID, "time-blocked decimator: C <= %d, q <= %d, N + 54 <= %d samples",
                              SB_MAXC, SB_MAXQ, SB_MAXT * SB_B);
        if (blocked)
            rc = fmt == TETRA_CF64 ? run_decimate_blocked<double>(ctx, P, (const double *)x, (int)C, (long)N,
                                                                  (double *)db, grouped(M))
                                   : run_decimate_blocked<float>(ctx, P, (const float *)x, (int)C, (long)N,
                                                                 (float *)db, grouped(M));
        else
            rc = fmt == TETRA_CF64 ? run_decimate<double>(ctx, P, (const double *)x, row_major(N), (int)C, (long)N,
                                                          (double *)db, grouped(M))
                                   : run_decimate<float>(ctx, P, (const float *)x, row_major(N), (int)C, (long)N,
                                                         (float *)db, grouped(M));
        if (rc) return rc;
        d = db;
        ld = grouped(M);
    }
    // stage 2: mixer + filtfilt (processor.py:260-264)
    const void *y = d;
    Lay ly = ld;
    bool y_f64 = fmt == TETRA_CF64;
    // latency mode (opt-in): the filtfilt passes time-blocked too (float64, ~1e-12 from scipy's
    // order); a few channels in any mode: extract_symbols' |y|^2 computed in parallel before its
    // per-phase sums (the same products and the same pairwise order: exact)
    const unsigned forms = compat_forms(P, C, N);
    if (P->filt || any_mix) {
        double *fb = (double *)ws(ctx, S_W3, grouped_elems((int)C, M) * 8);
        if (!fb) return TETRA_E_NOMEM;
        if (P->filt) {
            const bool lfb = forms & TETRA_FORM_LF_BLOCKED;
            if ((P->flags & TETRA_COMPAT_BLOCKED) && !lf_blocked_fits((int)C, M, P->ntaps))
                return tetra_fail(ctx, TETRA_E_INVALID, "time-blocked filtfilt: C <= %d, M + 30 <= %d samples",
                                  SB_MAXC, SB_MAXT * LB_B);
            if (lfb)
                rc = fmt == TETRA_CF64 ? run_filtfilt_blocked<double>(ctx, P, (const double *)d, ld, (int)C, M, mc, mo, fb,
                                                                      grouped(M))
                                       : run_filtfilt_blocked<float>(ctx, P, (const float *)d, ld, (int)C, M, mc, mo, fb,
                                                                     grouped(M));
            else if (premix_fits(C, mix_on)) {
                // a few channels, every one mixed: frequency_shift's values for the whole chunk in
                // parallel first (k_mix: the same mixed_val arithmetic, float64), then the sequential
                // filtfilt on them -- with the mixer inside its recursion one lane computed every
                // sample's float64 sincos in its dependent chain (3.98 of the 11.7 ms one-chunk call,
                // DESIGN §5.8).  The same values and the same double extension: bit-identical.
                double *pm = (double *)ws(ctx, S_W19, grouped_elems((int)C, M) * 8);
                if (!pm) return TETRA_E_NOMEM;
                {
                    PROF(ctx, "compat_mix");
                    if (fmt == TETRA_CF64)
                        hipLaunchKernelGGL(k_mix<double>, dim3(grid_for(C * M, 256)), dim3(256), 0, ctx->stream,
                                           (const double *)d, ld, (int)C, M, mc, mo, P->fs_dec, pm, grouped(M));
                    else
                        hipLaunchKernelGGL(k_mix<float>, dim3(grid_for(C * M, 256)), dim3(256), 0, ctx->stream,
                                           (const float *)d, ld, (int)C, M, mc, mo, P->fs_dec, pm, grouped(M));
                }
                rc = run_filtfilt<double>(ctx, P, pm, grouped(M), (int)C, M, nullptr, nullptr, fb, grouped(M));
            } else
                rc = fmt == TETRA_CF64 ? run_filtfilt<double>(ctx, P, (const double *)d, ld, (int)C, M, mc, mo, fb,
                                                              grouped(M))
                                       : run_filtfilt<float>(ctx, P, (const float *)d, ld, (int)C, M, mc, mo, fb,
                                                             grouped(M));
            if (rc) return rc;
        } else if (fmt == TETRA_CF64) {
            hipLaunchKernelGGL(k_mix<double>, dim3(grid_for(C * M, 256)), dim3(256), 0, ctx->stream, (const double *)d,
                               ld, (int)C, M, mc, mo, P->fs_dec, fb, grouped(M));
        } else {
            hipLaunchKernelGGL(k_mix<float>, dim3(grid_for(C * M, 256)), dim3(256), 0, ctx->stream, (const float *)d,
                               ld, (int)C, M, mc, mo, P->fs_dec, fb, grouped(M));
        }
        y = fb;
        ly = grouped(M);
        y_f64 = true;
    }
    // stage 3+4: extract_symbols + demodulate_dqpsk (processor.py:267-271)
    void *pw = nullptr;
    if (forms & TETRA_FORM_POW_PREPASS) {
        pw = ws(ctx, S_W18, (size_t)C * M * (y_f64 ? 8 : 4));
        if (!pw) return TETRA_E_NOMEM;
    }
    if (y_f64) {
        launch_extract<double>(ctx, (const double *)y, ly, (int)C, M, P->sps, P->phase_step, (double *)so, (long)smax, no,
                               nullptr, (double *)pw);
        launch_demod<double>(ctx, (const double *)so, (long)smax, (int)C, no, 0, P->thr, ho, (long)smax);
    } else {
        launch_extract<float>(ctx, (const float *)y, ly, (int)C, M, P->sps, P->phase_step, (float *)so, (long)smax, no,
                              nullptr, (float *)pw);
        launch_demod<float>(ctx, (const float *)so, (long)smax, (int)C, no, 0, P->thr, ho, (long)smax);
    }
    if (soft_f32) *soft_f32 = f32_soft ? 1 : 0;
    return st.finish();
}

}  // extern "C"
