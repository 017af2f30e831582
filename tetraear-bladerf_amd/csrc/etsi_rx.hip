// etsi_rx.hip -- ETSI EN 300 392-2 receive chain on gfx950 (the north-star path).
//
// The reference has no such chain; this is the receiver BASELINE.json's
// north_star asks for, restating oracle/etsi_oracle.c operation for operation (explicit fmaf,
// emulated 64-lane reductions, a libm-free atan2), so GPU and oracle results are bit-identical.
//
//   k_chanfilt_r stage 1: 48-tap decimate-by-10 FIR (2.4 MSps -> 240 kHz), stage 2: polyphase RRC
//                (alpha 0.35, 321 taps at 720 kHz) resampler x3/10 -> 72 kHz = 4 samples/symbol,
//                then the timing stage (fused).  cf32 (8 B/sample) and SC16 (4 B/sample) chunks up
//                to YLDS outputs: the workgroup's four waves stream the channel's quarters
//                independently (480-sample wave tiles, register prefetch, private LDS image and
//                stage-1 buffer; stage 1 in registers: a lane's 10-sample block from the image, the
//                next four blocks from its row neighbours by DPP folded into v_fmac_f32_dpp; stage 2
//                in one-MFMA-tile bursts on v_mfma_f32_16x16x4_f32 -- exact f32: banded tap matrix x
//                16 columns of 5 output triples), y held in LDS.
//   k_chanfilt   the same filter with workgroup-wide 2560-sample tiles (barrier per tile, stage 2
//                every 8 tiles): SC16 rows that are not a multiple of four samples (y round-tripped
//                through L2, four workgroups per CU) and chunks longer than YLDS outputs.
//   k_timing     one wave per channel: Oerder-Meyr timing phase (wave reduction), block Gardner
//                tracking (64 symbols per block = one per lane; error summed by xor-butterfly),
//                cubic interpolation, differential decision, 4th-power CFO estimate, int8 soft bits.
//   k_etsi_sync  one wave per channel: hard bits packed by ballots, head/training/tail correlation
//                by XOR+popcount, greedy burst scan, one decode job per coded block (dense atomic
//                allocation).
//   k_etsi_viterbi  four lanes per job: the block's type-5 soft bits loaded as dwords and
//                descrambled into an LDS row, deinterleave + depuncture applied on the trellis's
//                reads, 16-state rate-1/4 Viterbi with metrics in registers, survivors coalesced in
//                global scratch.
//   k_etsi_traceback  one lane per job: traceback with the CRC-16 folded in.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int ETSI_MAXB = 8;    // bursts per channel chunk
constexpr int ETSI_MAXJ = 16;   // coded blocks per channel chunk (2 per burst)
constexpr int TILE_K = 256;     // stage-1 outputs per tile (one per thread)
constexpr int TILE_IN = TILE_K * 10;   // new input samples per tile (q1 = 10)
constexpr int HALO = 48;

struct KindP { int K, a, n2, n1; };
__host__ __device__ constexpr KindP kind_params(int kind) {
    return kind == 0 ? KindP{432, 103, 288, 268} : kind == 1 ? KindP{216, 101, 144, 124} : KindP{120, 11, 80, 60};
}

// --------------------------------------------------------------------------- E2 timing
// 64-lane xor butterfly, levels 32, 16, .., LO: v_l + v_{l ^ off} at each level (the oracle's
// tree; fp add is commutative, so operand order within a pair is free).  Cross-lane moves stay in
// the VALU: permlane32/16 swaps for 32 and 16, DPP row rotations / quad permutes below (after the
// xor-8 level a lane's value depends only on l mod 8, so rotating a row by 4 reads l ^ 4's value,
// and by the same argument quad_perm covers 2 and 1) -- a ds_bpermute per level would put an LDS
// round trip on the Gardner loop's critical path.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    // bound_ctrl: a lane without a source reads 0 (only wave_shr's lane 0, which is replaced);
    // this form folds into the consuming v_add_f32_dpp
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int LO>
__device__ __forceinline__ float bfly(float v) {
    const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(b[0]) + __uint_as_float(b[1]);
    if constexpr (LO <= 8) v = v + dppf<0x128>(v);   // row_ror:8
    if constexpr (LO <= 4) v = v + dppf<0x124>(v);   // row_ror:4
    if constexpr (LO <= 2) v = v + dppf<0x4E>(v);    // quad_perm [2,3,0,1]
    if constexpr (LO <= 1) v = v + dppf<0xB1>(v);    // quad_perm [1,0,3,2]
    return v;
}
__device__ __forceinline__ float wave_sum(float v) { return bfly<1>(v); }
// two full butterflies level by level, interleaved: the Gardner block's error and power sums are
// one dependent chain each, and issued one after the other they doubled the loop's reduction latency
__device__ __forceinline__ void wave_sum2(float &u, float &v) {
    const auto a0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(u), __float_as_uint(u), false, false);
    const auto a1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    u = __uint_as_float(a0[0]) + __uint_as_float(a0[1]);
    v = __uint_as_float(a1[0]) + __uint_as_float(a1[1]);
    const auto b0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(u), __float_as_uint(u), false, false);
    const auto b1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    u = __uint_as_float(b0[0]) + __uint_as_float(b0[1]);
    v = __uint_as_float(b1[0]) + __uint_as_float(b1[1]);
    u = u + dppf<0x128>(u);
    v = v + dppf<0x128>(v);
    u = u + dppf<0x124>(u);
    v = v + dppf<0x124>(v);
    u = u + dppf<0x4E>(u);
    v = v + dppf<0x4E>(v);
    u = u + dppf<0xB1>(u);
    v = v + dppf<0xB1>(v);
}
__device__ __forceinline__ float lane_f(float v, int l) {   // wave-uniform l
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__device__ __forceinline__ float pat2(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float a = mx == 0.0f ? 0.0f : mn / mx;
    const float s = a * a;
    float r = fmaf(fmaf(fmaf(fmaf(fmaf(-0.0117212f, s, 0.05265332f), s, -0.11643287f), s, 0.19354346f), s,
                        -0.33262347f), s, 0.99997726f) * a;
    if (ay > ax) r = 1.57079637f - r;
    if (x < 0.0f) r = 3.14159274f - r;
    if (y < 0.0f) r = -r;
    return r;
}

// Cubic Lagrange interpolation of y (y[n] at w[n - w0]) at t and at t - 2 together: t - 2 is exact
// here (t < 2^22), so both share the fraction f and the four Lagrange weights -- computed once, the
// same bits either way.  (Measured and rejected: prefetching the next block's window at the position
// the current delta predicts, selected by the wave-uniform shift: 0.5 % slower -- the Gardner block is
// bound by its instruction chain, not by this LDS read.)
__device__ __forceinline__ void interp_pair(const float2 *w, int w0, float t, float2 &on, float2 &mid) {
    const float K6 = 1.0f / 6.0f;
    const float fi = floorf(t);
    const int i = (int)fi;
    const float f = t - fi;
    const float fm1 = f - 1.0f, fm2 = f - 2.0f, fp1 = f + 1.0f;
    const float cm = -(f * fm1 * fm2) * K6;
    const float c0 = (fp1 * fm1 * fm2) * 0.5f;
    const float c1 = -(fp1 * f * fm2) * 0.5f;
    const float c2 = (fp1 * f * fm1) * K6;
    auto one = [&](int j) -> float2 {
        const float2 a = w[j - 1 - w0], b = w[j - w0], c = w[j + 1 - w0], d = w[j + 2 - w0];
        float r = cm * a.x, q = cm * a.y;
        r = fmaf(c0, b.x, r); q = fmaf(c0, b.y, q);
        r = fmaf(c1, c.x, r); q = fmaf(c1, c.y, q);
        r = fmaf(c2, d.x, r); q = fmaf(c2, d.y, q);
        return make_float2(r, q);
    };
    on = one(i);
    mid = one(i - 2);
}

// interp_pair over a 512-sample LDS ring holding y[n] at ring[n & 511] (k_timing: the Gardner
// window staged from global memory a block ahead); the same operations as interp_pair
constexpr int TRING = 512;
__device__ __forceinline__ void interp_pair_ring(const float2 *w, float t, float2 &on, float2 &mid) {
    const float K6 = 1.0f / 6.0f;
    const float fi = floorf(t);
    const int i = (int)fi;
    const float f = t - fi;
    const float fm1 = f - 1.0f, fm2 = f - 2.0f, fp1 = f + 1.0f;
    const float cm = -(f * fm1 * fm2) * K6;
    const float c0 = (fp1 * fm1 * fm2) * 0.5f;
    const float c1 = -(fp1 * f * fm2) * 0.5f;
    const float c2 = (fp1 * f * fm1) * K6;
    auto one = [&](int j) -> float2 {
        const float2 a = w[(j - 1) & (TRING - 1)], b = w[j & (TRING - 1)], c = w[(j + 1) & (TRING - 1)],
                     d = w[(j + 2) & (TRING - 1)];
        float r = cm * a.x, q = cm * a.y;
        r = fmaf(c0, b.x, r); q = fmaf(c0, b.y, q);
        r = fmaf(c1, c.x, r); q = fmaf(c1, c.y, q);
        r = fmaf(c2, d.x, r); q = fmaf(c2, d.y, q);
        return make_float2(r, q);
    };
    on = one(i);
    mid = one(i - 2);
}

__device__ __forceinline__ float2 csqrt_p(float x, float y) {
    const float r = sqrtf(fmaf(x, x, y * y));
    if (r == 0.0f) return make_float2(0.f, 0.f);
    if (x >= 0.0f) {
        const float s = sqrtf((r + x) * 0.5f);
        return make_float2(s, y / (2.0f * s));
    }
    float s = sqrtf((r - x) * 0.5f);
    if (y < 0.0f) s = -s;
    return make_float2(y / (2.0f * s), s);
}

// The timing + decision stage for one channel.  timing_track runs on one wave (lane = 0..63): the
// Oerder-Meyr phase, block-Gardner tracking, and the CFO sums, which are folded into the Gardner
// blocks (lane l produces the symbols j = 64 b + l, ascending -- the order the oracle's CFO loop
// sums them in), so no second pass over d is needed; it leaves d_j in dp and returns the CFO
// rotation and soft scale.  timing_decide (the decision pass: rotation, int8 soft bits, hard
// dibits) is elementwise and is shared by `nw` waves.  y / dp may point to global memory (k_timing)
// or LDS (the fused demod); every cross-lane exchange in timing_track is a wave reduction or
// shuffle, so it needs no workgroup barrier.
struct TrackOut {
    int S;
    float rr, ri, sc, base, delta;
    int kstart, J0;   // first block's k; 1 when symbol 0 is the carried previous one (streaming)
    float pr, pi;     // the last symbol
};

// Streaming input of one channel's timing (tetra_etsi_track + the window's yoff): acq = 0 is the
// non-streaming receiver (Oerder-Meyr acquisition on the chunk, a new differential chain).
struct TrackIn {
    int acq;
    float base, delta, pr, pi;
    int yoff;
};
__device__ __forceinline__ TrackIn track_in(const tetra_etsi_track *t, int yoff) {
    if (!t) return TrackIn{0, 0.f, 0.f, 0.f, 0.f, 0};
    return TrackIn{t->acquired, t->base, t->delta, t->prev_re, t->prev_im, yoff};
}
// The state for the next chunk (oracle/etsi_oracle.c timing_core): the next symbol's base relative
// to this window's end, the loop offset and the last symbol.
__device__ __forceinline__ void track_store(tetra_etsi_track *t, const TrackIn &ti, const TrackOut &o, int M2) {
    if (M2 < 16) {
        if (ti.acq) t->base = ti.base + (float)(ti.yoff - M2);
        return;
    }
    if (ti.acq || o.S > 0) {
        t->base = o.base + (float)(4 * (o.kstart + o.S - o.J0) - M2);
        t->delta = o.delta;
        t->prev_re = o.pr;
        t->prev_im = o.pi;
        t->acquired = 1;
    }
}

constexpr int CPOL_SC1 = 16;   // gfx940+ cache-policy bits: sc0 1, nt 2, sc1 16 (copy_out)

// SPLIT: the CFO sums are left to a second wave (cfo_consumer) that follows the tracking through
// the LDS progress word *prog (symbols done | PROG_DONE at the end): off the serial tracking chain.
constexpr int PROG_DONE = 1 << 30;
// Oerder-Meyr part w for this lane: |y[n]|^2 summed over n = 64 b + lane, b in [w q4, (w + 1) q4),
// q4 = ceil(nb / 4) (loads issued 8 ahead; ascending order)
__device__ __forceinline__ float om_part(const float2 *y, int M2, int w, int lane) {
    const int nb = (M2 + 63) / 64, q4 = (nb + 3) / 4;
    const int n1 = min(64 * min((w + 1) * q4, nb), M2);
    float s = 0.f;
    for (int n0 = 64 * w * q4 + lane; n0 < n1; n0 += 8 * 64) {
        float2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = n0 + 64 * u < n1 ? y[n0 + 64 * u] : make_float2(0.f, 0.f);
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (n0 + 64 * u < n1) s += fmaf(v[u].x, v[u].x, v[u].y * v[u].y);
    }
    return s;
}
// The four om_part sums of one lane with the quarters' loads interleaved (k_timing, y in global
// memory): OM_U loads of each quarter in flight together -- 4 OM_U -- instead of om_part's 8 of one
// quarter, so the pass waits on 4x fewer round trips; each quarter still sums in ascending n and the
// quarters are added in order, so the result is om_part(0) + .. + om_part(3) to the bit.
constexpr int OM_U = 4;
__device__ __forceinline__ float om_all(const float2 *y, int M2, int lane) {
    const int nb = (M2 + 63) / 64, q4 = (nb + 3) / 4;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < q4; i += OM_U) {
        float2 v[4][OM_U];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int n1 = min(64 * min((w + 1) * q4, nb), M2);
#pragma unroll
            for (int u = 0; u < OM_U; ++u) {
                const int n = 64 * (w * q4 + i + u) + lane;
                v[w][u] = (i + u < q4 && n < n1) ? y[n] : make_float2(0.f, 0.f);
            }
        }
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int n1 = min(64 * min((w + 1) * q4, nb), M2);
#pragma unroll
            for (int u = 0; u < OM_U; ++u) {
                const int n = 64 * (w * q4 + i + u) + lane;
                if (i + u < q4 && n < n1) s[w] += fmaf(v[w][u].x, v[w][u].x, v[w][u].y * v[w][u].y);
            }
        }
    }
    return ((s[0] + s[1]) + s[2]) + s[3];
}

// RING (k_timing, y in global memory): the Gardner loop reads y from a 512-sample LDS ring (4 KB: eight
// one-wave workgroups per SIMD still fit) filled a block ahead -- block b needs y[4 kb - 5, 4 kb + 260)
// (|delta| <= 1.5, the cubic window), the ring holds [0, 320) before the loop, and block b first writes
// the 256 samples the previous block loaded into registers, [320 + 256 (b - 1), 320 + 256 b) (over
// [256 b - 448, 256 b - 192), which no later block reads), then loads the next 256: each block's window
// reads wait on LDS, not on L2 / HBM.  Same interpolation arithmetic, same bits.  RING = 2 keeps two
// blocks' loads in flight in registers (pre, pre2: the ring's contents at every block are the same).
// LEAN (k_timing): the Oerder-Meyr pass by om_all (all quarters' loads together) instead of om_part per
// quarter, and no d_j stores -- the decision pass recomputes d_j from the stored symbols (timing_decide_sym).
// OMC (k_timing's OMG form): the Oerder-Meyr class sums are given (omc = A0..A3, wave-uniform) --
// the wideband resampler formed their group partials -- and the pass over y is skipped.
template <bool SPLIT = false, int RING = 0, bool LEAN = false, bool OMC = false>
__device__ __forceinline__ TrackOut timing_track(const float2 *y, int M2, float gain, float soft_scale, float2 *sp,
                                                 float2 *dp, int smax, int lane, int *prog = nullptr,
                                                 const float *om = nullptr, float2 *ring = nullptr,
                                                 uint32_t *clk = nullptr, float4 omc = float4{},
                                                 TrackIn ti = TrackIn{}) {
    TrackOut o{0, 1.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0, 0, 0.0f, 0.0f};
    if (M2 < 16) {
        if constexpr (SPLIT) {
            if (lane == 0) __hip_atomic_store(prog, PROG_DONE, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return o;
    }
    // Oerder-Meyr: class sums of |y|^2 over n mod 4, per lane as four partial sums over quarters of
    // the blocks added in order (om_part; the oracle's order) -- precomputed by four waves (om)
    // or computed here one after the other.  Streaming with the loop acquired: no acquisition, the
    // carried base (plus the window's yoff) and delta continue (oracle timing_core)
    float A0 = 0.f, A1 = 0.f, A2 = 0.f, A3 = 0.f;
    if (ti.acq) {
    } else if constexpr (OMC) {
        A0 = omc.x;
        A1 = omc.y;
        A2 = omc.z;
        A3 = omc.w;
    } else {
        float s;
        if (om) {
            s = om[lane];
#pragma unroll
            for (int w = 1; w < 4; ++w) s = s + om[64 * w + lane];
        } else if constexpr (LEAN) {
            s = om_all(y, M2, lane);
        } else {
            s = om_part(y, M2, 0, lane);
#pragma unroll
            for (int w = 1; w < 4; ++w) s = s + om_part(y, M2, w, lane);
        }
        s = bfly<4>(s);
        A0 = lane_f(s, 0);
        A1 = lane_f(s, 1);
        A2 = lane_f(s, 2);
        A3 = lane_f(s, 3);
    }
    if (clk && lane == 0) clk[1] = (uint32_t)wall_clock64();   // probe: the Oerder-Meyr pass done
    float base, delta;
    int kstart;
    const int J0 = ti.acq ? 1 : 0;
    if (ti.acq) {
        base = ti.base + (float)ti.yoff;
        delta = ti.delta;
        kstart = 0;
    } else {
        const float Xr = A0 - A2, Xi = A3 - A1;
        const float p = -0.63661977236758134f * pat2(Xi, Xr);
        base = p < 0.0f ? p + 4.0f : p;
        if (base >= 4.0f) base -= 4.0f;
        kstart = base >= 3.0f ? 0 : 1;
        delta = 0.0f;
    }
    int S = J0;   // symbol 0 of a continued stream is the carried last symbol
    float2 prev = J0 ? make_float2(ti.pr, ti.pi) : make_float2(0.f, 0.f);
    bool have_prev = J0 != 0;
    if (J0 && lane == 0 && smax > 0) sp[0] = prev;
    float zr = 0.f, zi = 0.f, am = 0.f;   // CFO sums over this lane's d_j
    int rel = -1;   // SPLIT: progress not yet released (published after the next block's LDS reads)
    float2 pre[4], pre2[4];   // RING: the next block's 256 samples in flight (RING 2: and the one after)
    // RING: the ring's loads go through a buffer resource over y (past M2 they return 0) and the symbol
    // stores through one over sp (past smax they are dropped), both without branches: hipcc then
    // counts the wave's memory operations exactly and waits at a block's ring writes only for the
    // loads it needs, not (vmcnt(0)) for the previous block's symbol stores as well
    typedef unsigned u2v __attribute__((ext_vector_type(2)));
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2 *>(y), 0, 8 * M2, 0x00020000);
    const __amdgpu_buffer_rsrc_t sps = __builtin_amdgcn_make_buffer_rsrc(sp, 0, 8 * smax, 0x00020000);
    auto ld = [&](int n) -> float2 {
        if constexpr (RING > 0) {
            const u2v v = __builtin_amdgcn_raw_buffer_load_b64(yrs, 8 * n, 0, 0);
            return make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
        } else {
            return n < M2 ? y[n] : make_float2(0.f, 0.f);
        }
    };
    if constexpr (RING > 0) {
#pragma unroll
        for (int u = 0; u < 5; ++u) ring[64 * u + lane] = ld(64 * u + lane);
#pragma unroll
        for (int u = 0; u < 4; ++u) pre[u] = ld(320 + 64 * u + lane);
        if constexpr (RING > 1) {
#pragma unroll
            for (int u = 0; u < 4; ++u) pre2[u] = ld(576 + 64 * u + lane);
        }
    }
    for (int kb = kstart;; kb += 64) {
        if constexpr (RING > 0) {
            if (kb != kstart) {   // the previous block's loads: y[320 + 256 (b - 1) ...)
                const int n0 = 320 + 4 * (kb - kstart) - 256;
#pragma unroll
                for (int u = 0; u < 4; ++u) ring[(n0 + 64 * u + lane) & (TRING - 1)] = pre[u];
                if constexpr (RING > 1) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        pre[u] = pre2[u];
                        pre2[u] = ld(n0 + 512 + 64 * u + lane);
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u) pre[u] = ld(n0 + 256 + 64 * u + lane);
                }
            }
        }
        const float off = base + delta;
        const float t = (float)(4 * (kb + lane)) + off;
        const bool valid = (t - 3.0f >= 0.0f) && (t + 2.0f <= (float)(M2 - 1)) && (S + lane < smax);
        const unsigned long long bal = __ballot(!valid);
        const int nv = bal ? (__ffsll((long long)bal) - 1) : 64;
        const bool act = lane < nv;
        float2 on = make_float2(0.f, 0.f), mid = make_float2(0.f, 0.f);
        if constexpr (SPLIT) {
            // y in LDS: every lane interpolates, so the window reads do not wait for the ballot
            // (a lane past nv reads in or past the workgroup's LDS -- past it reads return 0 -- and
            // its values are dropped below)
            float2 a, b;
            interp_pair(y, 0, t, a, b);
            asm volatile("" ::"v"(a.x), "v"(a.y), "v"(b.x), "v"(b.y));   // computed here, not sunk into the branch
            if (act) {
                on = a;
                mid = b;
            }
            if (rel >= 0 && lane == 0)   // the previous block's d_j: its stores completed before these reads
                __hip_atomic_store(prog, rel, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if constexpr (RING > 0) {
            if (act) interp_pair_ring(ring, t, on, mid);
        } else {
            if (act) interp_pair(y, 0, t, on, mid);
        }
        float2 pv = make_float2(dppf<0x138>(on.x), dppf<0x138>(on.y));   // wave_shr:1 (lane 0 replaced below)
        bool hp_ = true;
        if (lane == 0) { pv = prev; hp_ = have_prev; }
        float ev = 0.f, pw = 0.f;
        if (act) {
            pw = fmaf(on.x, on.x, on.y * on.y);
            if (hp_) {
                const float dr = on.x - pv.x, di = on.y - pv.y;
                ev = fmaf(dr, mid.x, di * mid.y);
                const int j = S + lane;
                const float xr = fmaf(on.x, pv.x, on.y * pv.y), xi = fmaf(on.y, pv.x, -(on.x * pv.y));
                if constexpr (!LEAN) dp[j - 1] = make_float2(xr, xi);
                if constexpr (!SPLIT) {
                    // CFO: 4th power and magnitude of d_j (j = lane mod 64, ascending: the oracle's order)
                    const float sr = fmaf(xr, xr, -(xi * xi)), si = (xr * xi) * 2.0f;
                    const float qr = fmaf(sr, sr, -(si * si)), qi = (sr * si) * 2.0f;
                    zr += qr;
                    zi += qi;
                    am += sqrtf(fmaf(xr, xr, xi * xi));
                }
            }
            if constexpr (RING == 0) sp[S + lane] = on;
        }
        // RING: every lane stores (a lane past nv stores 0 at S + lane >= the final S, or nothing past smax)
        if constexpr (RING > 0)
            __builtin_amdgcn_raw_buffer_store_b64(u2v{__float_as_uint(on.x), __float_as_uint(on.y)}, sps, 8 * (S + lane),
                                                  0, 0);
        if (nv > 0) {
            float E = ev, W = pw;
            wave_sum2(E, W);
            if (W > 0.0f) delta = delta - gain * (E / W);
            if (delta > 1.5f) delta = 1.5f;
            if (delta < -1.5f) delta = -1.5f;
            prev = make_float2(lane_f(on.x, nv - 1), lane_f(on.y, nv - 1));
            have_prev = true;
        }
        S += nv;
        if constexpr (SPLIT) rel = S;   // d_j, j < S, are in dp: released to the CFO wave next block
        if (nv < 64) break;
    }
    if constexpr (SPLIT) {   // the last block's d_j, and the end
        if (lane == 0) __hip_atomic_store(prog, S | PROG_DONE, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    o.S = S;
    o.base = base;
    o.delta = delta;
    o.kstart = kstart;
    o.J0 = J0;
    o.pr = prev.x;
    o.pi = prev.y;
    if constexpr (SPLIT) return o;   // rr, ri, sc: cfo_consumer's
    // CFO rotation conj((-Z/|Z|)^(1/4)) and the soft scale from the mean |d|
    const float Zr = wave_sum(zr), Zi = wave_sum(zi), A = wave_sum(am);
    float rr = 1.0f, ri = 0.0f;
    const float zm = sqrtf(fmaf(Zr, Zr, Zi * Zi));
    if (zm > 0.0f) {
        const float2 v = csqrt_p(-Zr / zm, -Zi / zm);
        const float2 w = csqrt_p(v.x, v.y);
        rr = w.x;
        ri = -w.y;
    }
    o.rr = rr;
    o.ri = ri;
    o.sc = (S > 1 && A > 0.0f) ? soft_scale / (A / (float)(S - 1)) : 0.0f;
    return o;
}

// The CFO half of timing_track<false>, on a second wave while timing_track<true> tracks: lane l
// sums the 4th powers and magnitudes of d_j, j = l mod 64, block after block as the progress word
// releases them -- the same per-lane order, so the same bits -- then the rotation and the soft
// scale into *o (rr, ri, sc).
__device__ __forceinline__ void cfo_consumer(const float2 *dp, float soft_scale, int *prog, TrackOut *o, int lane,
                                             int j0 = 0) {
    // lane l sums d_j for j = j0 + l mod 64 (j0 = 1 when symbol 0 is a continued stream's carried one):
    // the tracking wave's lane order
    float zr = 0.f, zi = 0.f, am = 0.f;
    int jb = j0, S = 0;
    for (;;) {
        const int v = __hip_atomic_load(prog, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        S = v & (PROG_DONE - 1);
        for (; jb < S; jb += 64) {
            const int j = jb + lane;
            if (j >= 1 && j < S) {
                const float2 d = dp[j - 1];
                const float xr = d.x, xi = d.y;
                const float sr = fmaf(xr, xr, -(xi * xi)), si = (xr * xi) * 2.0f;
                const float qr = fmaf(sr, sr, -(si * si)), qi = (sr * si) * 2.0f;
                zr += qr;
                zi += qi;
                am += sqrtf(fmaf(xr, xr, xi * xi));
            }
        }
        if (v & PROG_DONE) break;
        __builtin_amdgcn_s_sleep(1);
    }
    const float Zr = wave_sum(zr), Zi = wave_sum(zi), A = wave_sum(am);
    float rr = 1.0f, ri = 0.0f;
    const float zm = sqrtf(fmaf(Zr, Zr, Zi * Zi));
    if (zm > 0.0f) {
        const float2 v = csqrt_p(-Zr / zm, -Zi / zm);
        const float2 w = csqrt_p(v.x, v.y);
        rr = w.x;
        ri = -w.y;
    }
    if (lane == 0) {
        o->rr = rr;
        o->ri = ri;
        o->sc = (S > 1 && A > 0.0f) ? soft_scale / (A / (float)(S - 1)) : 0.0f;
    }
}

// Decision pass over d_j, j in [1, S): wave w of nw takes the 64-symbol blocks w, w + nw, ...
__device__ __forceinline__ void timing_decide(const TrackOut &o, const float2 *dp, int8_t *sb, uint8_t *hp, int w,
                                              int nw, int lane) {
    for (int j0 = 1 + 64 * w + lane; j0 < o.S; j0 += 4 * 64 * nw) {
        float2 dv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) dv[u] = j0 + 64 * nw * u < o.S ? dp[j0 + 64 * nw * u - 1] : make_float2(0.f, 0.f);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + 64 * nw * u;
            if (j >= o.S) break;
            const float2 d = dv[u];
            const float xr = fmaf(d.x, o.rr, -(d.y * o.ri)), xi = fmaf(d.x, o.ri, d.y * o.rr);
            float q1 = rintf(xi * o.sc), q2 = rintf(xr * o.sc);
            q1 = q1 > 127.f ? 127.f : (q1 < -127.f ? -127.f : q1);
            q2 = q2 > 127.f ? 127.f : (q2 < -127.f ? -127.f : q2);
            sb[2 * (j - 1)] = (int8_t)q1;
            sb[2 * (j - 1) + 1] = (int8_t)q2;
            hp[j - 1] = (uint8_t)(((xi < 0.0f) << 1) | (xr < 0.0f));
        }
    }
}

// timing_decide with d_j = s_j conj(s_{j-1}) recomputed from the stored symbols sp -- the same fmas on
// the same values the tracking loop formed it from, so the same bits (k_timing LEAN: d_j is not stored)
__device__ __forceinline__ void timing_decide_sym(const TrackOut &o, const float2 *sp, int8_t *sb, uint8_t *hp,
                                                  int lane) {
    for (int j0 = 1 + lane; j0 < o.S; j0 += 4 * 64) {
        float2 a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + 64 * u;
            a[u] = j < o.S ? sp[j] : make_float2(0.f, 0.f);
            b[u] = j < o.S ? sp[j - 1] : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + 64 * u;
            if (j >= o.S) break;
            const float2 on = a[u], pv = b[u];
            const float dx = fmaf(on.x, pv.x, on.y * pv.y), dy = fmaf(on.y, pv.x, -(on.x * pv.y));
            const float xr = fmaf(dx, o.rr, -(dy * o.ri)), xi = fmaf(dx, o.ri, dy * o.rr);
            float q1 = rintf(xi * o.sc), q2 = rintf(xr * o.sc);
            q1 = q1 > 127.f ? 127.f : (q1 < -127.f ? -127.f : q1);
            q2 = q2 > 127.f ? 127.f : (q2 < -127.f ? -127.f : q2);
            sb[2 * (j - 1)] = (int8_t)q1;
            sb[2 * (j - 1) + 1] = (int8_t)q2;
            hp[j - 1] = (uint8_t)(((xi < 0.0f) << 1) | (xr < 0.0f));
        }
    }
}

// clk (probe, TETRA_TIMING_PROBE=1 with a diag buffer): the wave's wall-clock stamps at its start, after
// the Oerder-Meyr pass, after the Gardner loop and at its end, in place of the diagnostics
template <int RING = 0, bool LEAN = false, bool OMC = false>
__device__ __forceinline__ void timing_wave(const float2 *y, int M2, float gain, float soft_scale, float2 *sp,
                                            float2 *dp, int8_t *sb, uint8_t *hp, int32_t *nsym_ch, float4 *diag_ch,
                                            int smax, int lane, float2 *ring = nullptr, uint32_t *clk = nullptr,
                                            float4 omc = float4{}, tetra_etsi_track *trk = nullptr, int yoff = 0) {
    if (!OMC && clk && lane == 0) clk[0] = (uint32_t)wall_clock64();   // OMC: stamped before the class sums
    const TrackIn ti = track_in(trk, yoff);
    const TrackOut o = timing_track<false, RING, LEAN, OMC>(y, M2, gain, soft_scale, sp, dp, smax, lane, nullptr,
                                                            nullptr, ring, clk, omc, ti);
    if (trk && lane == 0) track_store(trk, ti, o, M2);
    if (clk && lane == 0) clk[2] = (uint32_t)wall_clock64();
    __threadfence_block();   // dp / sp written by other lanes is read below
    if constexpr (LEAN)
        timing_decide_sym(o, sp, sb, hp, lane);
    else
        timing_decide(o, dp, sb, hp, 0, 1, lane);
    if (lane == 0) {
        *nsym_ch = o.S;
        if (clk) {
            __builtin_amdgcn_s_waitcnt(0);   // the decision pass's stores issued and done
            clk[3] = (uint32_t)wall_clock64();
        } else if (diag_ch && M2 >= 16) {
            *diag_ch = make_float4(o.base, o.delta, o.rr, o.ri);
        }
    }
}

// The Oerder-Meyr class sums of the chunk row[s, e) in the wideband grouped order (oracle
// eo_om_grouped): P holds the carrier row's resampler group partials (U outputs per group, s a
// multiple of 4).  Lane l sums the whole groups g0 + l, g0 + l + 64, ... then a wave butterfly; the
// head [s, U g0) and the tail [U g1, e) (each < U <= 64 samples, one per lane) are summed class by
// class in ascending n.
__device__ __forceinline__ float4 om_grouped(const float2 *__restrict__ row, const float4 *__restrict__ P, long s,
                                             long e, int U, int lane) {
    const long g0 = (s + U - 1) / U, g1 = e / U;
    const long hend = min((long)U * g0, e), tbeg = max((long)U * g1, hend);
    // head and tail samples first (their loads in flight with the partials')
    const long hi = s + lane, ti = tbeg + lane;
    const float2 hv = hi < hend ? row[hi] : make_float2(0.f, 0.f);
    const float2 tv = ti < e ? row[ti] : make_float2(0.f, 0.f);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    for (long g = g0 + lane; g < g1; g += 64) {
        const float4 p = P[g];
        v.x = v.x + p.x;
        v.y = v.y + p.y;
        v.z = v.z + p.z;
        v.w = v.w + p.w;
    }
    const float ph = fmaf(hv.x, hv.x, hv.y * hv.y), pt = fmaf(tv.x, tv.x, tv.y * tv.y);
    wave_sum2(v.x, v.y);
    wave_sum2(v.z, v.w);
    float h[4] = {0.f, 0.f, 0.f, 0.f}, t[4] = {0.f, 0.f, 0.f, 0.f};
    const int nh = (int)(hend - s), nt = (int)(e - tbeg);   // < U <= 64
    for (int i = 0; i < nh; ++i) h[i & 3] = h[i & 3] + lane_f(ph, i);
    for (int i = 0; i < nt; ++i) t[i & 3] = t[i & 3] + lane_f(pt, i);
    return make_float4((h[0] + v.x) + t[0], (h[1] + v.y) + t[1], (h[2] + v.z) + t[2], (h[3] + v.w) + t[3]);
}

// Chunked rows (cstride > 0: tetra_etsi_timing_chunks / _om): block ch is chunk c = ch mod nchunk of
// carrier k = ch / nchunk, the samples yall[k rowlen + c cstride, ...) up to M2 of them or the row's
// end (chunks may overlap); cstride = 0: block ch is yall[ch M2, (ch + 1) M2).
// OMG (the _om forms): the Oerder-Meyr class sums from the resampler's group partials (om: ngrp
// float4 per carrier row)
template <int RING, bool LEAN, bool OMG = false>
__global__ __launch_bounds__(64) void k_timing(const float2 *__restrict__ yall, int M2, float gain, float soft_scale,
                                               float2 *__restrict__ sym, float2 *__restrict__ dscr,
                                               int8_t *__restrict__ softbits, uint8_t *__restrict__ hard,
                                               int32_t *__restrict__ nsym, int smax, float4 *__restrict__ diag,
                                               int probe, const float4 *__restrict__ om, int nchunk, int ngrp, int U,
                                               tetra_etsi_track *__restrict__ trk, int yoff, int ostride, int cstride,
                                               long rowlen) {
    __shared__ float2 ring[RING ? TRING : 1];
    const int ch = blockIdx.x;
    uint32_t *clk = probe && diag ? reinterpret_cast<uint32_t *>(diag + ch) : nullptr;
    const float2 *y = yall + (size_t)ch * M2;
    int L = M2;
    float4 omc = float4{};
    if (cstride > 0) {
        const int k = ch / nchunk;
        const long s = (long)(ch - k * nchunk) * cstride;
        L = (int)min((long)M2, rowlen - s);
        const float2 *row = yall + (size_t)k * rowlen;
        y = row + s;
        if constexpr (OMG) {
            if (clk && threadIdx.x == 0) clk[0] = (uint32_t)wall_clock64();
            omc = om_grouped(row, om + (size_t)k * ngrp, s, s + L, U, threadIdx.x);
        }
    }
    const size_t os = ostride ? (size_t)ostride : (size_t)smax;   // output rows (streaming: reserve + smax)
    timing_wave<RING, LEAN, OMG>(y, L, gain, soft_scale, sym + (size_t)ch * os,
                                 dscr ? dscr + (size_t)ch * smax : nullptr, softbits + (size_t)ch * 2 * os,
                                 hard + (size_t)ch * os, nsym + ch, diag ? diag + ch : nullptr, smax, threadIdx.x, ring,
                                 clk, omc, trk ? trk + ch : nullptr, yoff);
}
// k_timing's form (same-box A/B): TETRA_TIMING_RING = 0 (the Gardner windows read straight from
// global memory), 1 (one block ahead, default) or 2 (two); TETRA_TIMING_LEAN = 0 keeps om_part per
// quarter for the Oerder-Meyr pass and the d_j round trip through dscr (default 1: om_all, d_j
// recomputed from the symbols)
using timing_fn = void (*)(const float2 *, int, float, float, float2 *, float2 *, int8_t *, uint8_t *, int32_t *, int,
                           float4 *, int, const float4 *, int, int, int, tetra_etsi_track *, int, int, int, long);
// TETRA_TIMING_PROBE=1: with a diag buffer, each chunk's diag entry holds four 32-bit wall-clock stamps
// (start, Oerder-Meyr done, Gardner done, end) instead of the diagnostics -- a latency probe
static int timing_probe() {
    const char *e = getenv("TETRA_TIMING_PROBE");
    return e && atoi(e) == 1;
}
static timing_fn timing_kernel(size_t M2, size_t smax, bool omg = false) {
    const char *r = getenv("TETRA_TIMING_RING"), *o = getenv("TETRA_TIMING_LEAN");
    // the ring form addresses y and the symbols through buffer resources (32-bit byte ranges)
    const bool fits = 8 * M2 < ((size_t)1 << 31) && 8 * smax < ((size_t)1 << 31);
    const int ring = !fits ? 0 : (r ? atoi(r) : 1);
    const bool lean = !(o && atoi(o) == 0);
    if (omg) return ring <= 0 ? k_timing<0, true, true> : k_timing<1, true, true>;
    if (ring <= 0) return lean ? k_timing<0, true> : k_timing<0, false>;
    if (ring == 1) return lean ? k_timing<1, true> : k_timing<1, false>;
    return lean ? k_timing<2, true> : k_timing<2, false>;
}

// --------------------------------------------------------------------------- E1 channel filter
// The input tile is a linear float4 image (2 samples per entry, ds_write_b128 / ds_read_b128: a
// 20-dword lane stride is conflict-free for b128's lane groups).  Stage-1 outputs x240[k] go to a
// linear buffer lin[k - kbase]; after each stage-2 burst the still-needed tail is moved to its
// front (kbase = 10 u_done), so stage 2's operand reads are base + immediate offset.
// Stage 2 runs every S2_EVERY tiles (~205 output triples at 8).  Measured for cf32 (same box):
// serial demod every 12 tiles (LR 3336, 79.6 KB) 0.8 % faster than every 8 (1.569 vs 1.581 ms;
// 10 and 8 equal, 6 and 4 slower), but the pipelined step 0.7 % slower (1.694 vs 1.683 ms): at
// 2 x 79.6 KB the CU has no LDS left for the lower MAC's 7 KB workgroups, which then wait for a
// demod workgroup to retire.  The bench's pipelined step decides: 8 (16 KB free per CU).
template <typename In> struct CfCfg;
template <> struct CfCfg<float4> { static constexpr int s2_every = 8, lr = 2312; };
template <> struct CfCfg<uint2> { static constexpr int s2_every = 8, lr = 2312; };
constexpr int TPP = 107;        // RRC taps per polyphase branch (Lp = 321 = 3 x 107)
constexpr int PFD = 2;          // k_chanfilt: input tiles in flight per workgroup (register prefetch
                                // depth, pa/pb; 3 and 4 measured no faster)
constexpr int YLDS = 3968;      // cf32: stage-2 outputs held in LDS (a 131072-sample chunk has 3899; a
                                // streaming window of one, the previous chunk's last samples included, <= 3945)
// Stage 2 on the matrix cores (v_mfma_f32_16x16x4_f32: bit-for-bit a k-ordered fmaf chain).  One
// MFMA tile: 16 columns = 8 segments x (re, im), each segment S2Q consecutive triples; row
// i = 3q + c of a column is output 3(U + q) + c; A[i][s] = tap of x240[10U + s] for that output
// (zero outside its 107: leading zeros keep the accumulator +0, trailing ones add +-0), so every
// output is the oracle's ascending-j fma chain.
constexpr int S2Q = 5;          // triples per column (rows 0..14; row 15 all-zero taps)
constexpr int S2T = 8 * S2Q;    // triples per MFMA tile
constexpr int S2K = 39;         // k-steps of 4: window 10 (S2Q - 1) + 114 = 154 -> 156 stage-1 outputs
// linear stage-1 buffer (float2): S2_EVERY tiles of 256 outputs + the next triples' windows
template <typename In> constexpr int cf_lr() { return CfCfg<In>::lr; }
constexpr int XIN4 = (HALO + TILE_IN) / 2;   // float4 entries of the input image
template <typename In> constexpr int cf_lds4() { return XIN4 + cf_lr<In>() / 2; }   // image + stage-1 buffer (float4)
constexpr int CF_LDS2_SC16 = 2 * (XIN4 + CfCfg<uint2>::lr / 2);   // SC16 fused: y + timing scratch (float2)
static_assert(XIN4 + CfCfg<uint2>::lr / 2 == 2460, "SC16 LDS: 39,360 B, four workgroups per CU");
static_assert((XIN4 + CfCfg<float4>::lr / 2 + 12) * 16 + 4096 * 8 <= 72 * 1024, "cf32 LDS: two workgroups per CU + 16 KB");
constexpr int CF_COEF = 128 + S2K * 64;      // device tap image: h1 (64), h1 * 2^-15 (64, SC16) + A fragments [S2K][64 lanes]

// Packed fp32 (v_pk_fma_f32): one real tap times a complex sample, each half a correctly rounded
// fma -- the same per-component arithmetic as two fmaf calls.
typedef float pf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pf2 pfma(float h, pf2 x, pf2 acc) { return __builtin_elementwise_fma(pf2{h, h}, x, acc); }
typedef float f4 __attribute__((ext_vector_type(4)));

// h1[48] stage-1 taps (wave-uniform, scalar loads); stage 2: branch c, output m = 3u + c =
// sum_j hp[i0(c) - 3j] * x240[10u + off_c + j] with i0 = {320, 318, 319}, off_c = {0, 4, 7}, held
// as the MFMA A fragments (one VGPR per k-step per lane, loaded once).
// Input pairs: one load = two complex samples -- float4 for cf32, uint2 (4 x int16) for SC16, the
// BladeRF wire format (capture.py:241-269 scales by 1/32768, exact in fp32), so an SC16 capture is
// filtered straight from its 4 B/sample form.
__device__ __forceinline__ float4 pair_f32(float4 v) { return v; }
__device__ __forceinline__ float4 pair_f32(uint2 v) {
    constexpr float s = 1.0f / 32768.0f;
    return make_float4((float)(int16_t)(v.x & 0xffffu) * s, (float)(int16_t)(v.x >> 16) * s,
                       (float)(int16_t)(v.y & 0xffffu) * s, (float)(int16_t)(v.y >> 16) * s);
}

// Timing outputs of the fused demod (FUSE = true: y never leaves LDS; wave 0 runs the timing
// stage on it after the last tile, with the input image as its scratch).
struct TimingOut {
    float gain, soft_scale;
    float2 *sym;
    int8_t *softbits;
    uint8_t *hard;
    int32_t *nsym;
    float4 *diag;
    int smax;
    int probe;   // TETRA_TIMING_PROBE: diag holds wall-clock stamps (start, tail start, tracking done, end)
    int ostride;                // row stride of sym / hard (softbits: 2x) -- 0: smax (streaming: reserve + smax)
    int yoff;                   // streaming: the window index of the first new 72 kHz output
    tetra_etsi_track *track;    // streaming: the channels' timing state (in/out), or null
};

// LDS -> global copy of n bytes by the workgroup's 256 threads, as device-scope (sc1) stores
// through a buffer resource over the row: 16-B stores where the row is 16-B aligned (the LDS image
// is), 8-B stores where it is 8-B aligned, byte stores for the rest.  sc1 writes the lines through
// to memory as they are stored; with the default policy the dirty lines sit in L2 and are evicted
// one by one into the channel filter's read stream (same box: demod 1.500 -> 1.423-1.437 ms; nt
// stores no better than the default; sc0 sc1 / nt sc1 / sc0 sc1 nt 1.43-1.45).
__device__ __forceinline__ void copy_out(uint8_t *g, const uint8_t *l, int n, int tid) {
    if (n <= 0) return;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(g, 0, n, 0x00020000);   // n: the range check
    const uintptr_t al = reinterpret_cast<uintptr_t>(g);
    int done = 0;
    if ((al & 15) == 0) {
        typedef unsigned u4v __attribute__((ext_vector_type(4)));
        const int n16 = n >> 4;
        for (int i = tid; i < n16; i += 256) {
            const uint4 v = reinterpret_cast<const uint4 *>(l)[i];
            __builtin_amdgcn_raw_buffer_store_b128(u4v{v.x, v.y, v.z, v.w}, r, 16 * i, 0, CPOL_SC1);
        }
        done = 16 * n16;
    } else if ((al & 7) == 0) {
        typedef unsigned u2v __attribute__((ext_vector_type(2)));
        const int n8 = n >> 3;
        for (int i = tid; i < n8; i += 256) {
            const uint2 v = reinterpret_cast<const uint2 *>(l)[i];
            __builtin_amdgcn_raw_buffer_store_b64(u2v{v.x, v.y}, r, 8 * i, 0, CPOL_SC1);
        }
        done = 8 * n8;
    }
    for (int i = done + tid; i < n; i += 256) __builtin_amdgcn_raw_buffer_store_b8(l[i], r, i, 0, CPOL_SC1);
}

// Output staging of the fused demod's tail (stage != nullptr): the symbols, soft bits and hard
// dibits of the channel collect in LDS and leave in wide stores once the channel is decided --
// per-block float2 stores from the tracking loop and byte stores from the decision pass cost
// 0.155 ms per 8192-channel batch (same box: 1.505 -> 1.350 ms with the stores left out).
struct TailStage {
    float2 *sym;     // [sm] (LDS)
    int8_t *sb;      // [2 sm]
    uint8_t *hard;   // [sm]
};

// The fused demod's timing stage for channel ch on y in LDS (ly), after the workgroup's last barrier:
// the tracking is the serial tail (wave 0, prioritised on its SIMD); the decision pass after it is
// shared by all four waves (the rotation and scale go through LDS, *tro).
__device__ __forceinline__ void timing_tail(const float2 *ly, float2 *scr, const TimingOut &to, int M2, int ch,
                                            int tid, TrackOut *tro, int *prog, const TailStage *stage = nullptr,
                                            float *om = nullptr, uint32_t t0 = 0) {
    const size_t so = (size_t)ch * (to.ostride ? to.ostride : to.smax);
    const bool probe = to.probe && to.diag;
    uint32_t t1 = 0, t2 = 0;
    if (probe && tid == 0) t1 = (uint32_t)wall_clock64();
    const TrackIn ti = track_in(to.track ? to.track + ch : nullptr, to.yoff);
    // the four Oerder-Meyr parts at once (not for a continued stream: no acquisition)
    if (om && M2 >= 16 && !ti.acq) om[tid] = om_part(ly, M2, tid >> 6, tid & 63);
    if (tid == 0) *prog = 0;
    __syncthreads();
    if (tid < 64) {
        __builtin_amdgcn_s_setprio(3);
        // S <= M2 / 4 + 1 < the staging size either way: the bound only guards the LDS buffer
        const TrackOut o = timing_track<true>(ly, M2, to.gain, to.soft_scale, stage ? stage->sym : to.sym + so, scr,
                                              stage ? min(to.smax, M2 / 4 + 3) : to.smax, tid, prog, om, nullptr,
                                              nullptr, float4{}, ti);
        if (tid == 0) {
            tro->S = o.S;
            tro->base = o.base;
            tro->delta = o.delta;
            to.nsym[ch] = o.S;
            if (to.track) track_store(to.track + ch, ti, o, M2);
            if (probe) t2 = (uint32_t)wall_clock64();
        }
    } else if (tid < 128) {
        cfo_consumer(scr, to.soft_scale, prog, tro, tid & 63, ti.acq ? 1 : 0);
    }
    __syncthreads();
    const TrackOut o = *tro;
    if (tid == 0 && to.diag && M2 >= 16 && !probe) to.diag[ch] = make_float4(o.base, o.delta, o.rr, o.ri);
    auto stamp = [&]() {
        if (probe && tid == 0) {
            __builtin_amdgcn_s_waitcnt(0);
            const uint32_t t3 = (uint32_t)wall_clock64();
            to.diag[ch] = make_float4(__uint_as_float(t0), __uint_as_float(t1), __uint_as_float(t2), __uint_as_float(t3));
        }
    };
    if (!stage) {
        timing_decide(o, scr, to.softbits + 2 * so, to.hard + so, tid >> 6, 4, tid & 63);
        stamp();
        return;
    }
    timing_decide(o, scr, stage->sb, stage->hard, tid >> 6, 4, tid & 63);
    __syncthreads();
    const int nd = o.S > 1 ? o.S - 1 : 0;
    copy_out(reinterpret_cast<uint8_t *>(to.sym + so), reinterpret_cast<const uint8_t *>(stage->sym), 8 * o.S, tid);
    copy_out(reinterpret_cast<uint8_t *>(to.softbits + 2 * so), reinterpret_cast<const uint8_t *>(stage->sb), 2 * nd,
             tid);
    copy_out(to.hard + so, stage->hard, nd, tid);
    stamp();
}

// SC16 is held to 128 VGPRs: four workgroups per CU (its LDS allows four; at 158-161 VGPRs it ran at
// three, 1.10 -> 1.57 ms per batch)
template <typename In> constexpr int cf_waves() { return std::is_same<In, float4>::value ? 2 : 4; }
template <typename In, bool FUSE>
__global__ __launch_bounds__(256, cf_waves<In>()) void k_chanfilt(const In *__restrict__ iq, long N, int M1, int M2,
                                                  const float *__restrict__ h1, const float *__restrict__ afrag,
                                                  float2 *__restrict__ y, TimingOut to, long ld) {
    constexpr bool YL = std::is_same<In, float4>::value;
    // cf32 keeps y in LDS (yb, 72 KB: two workgroups per CU, no y traffic); SC16 streams half the
    // bytes per sample and is bound by the workgroup's own LDS/issue chain instead, so it keeps
    // only the image and the stage-1 buffer (39 KB: four workgroups per CU) and sends y through
    // HBM/L2
    constexpr int CF_LDS4 = cf_lds4<In>(), LR = cf_lr<In>(), S2_EVERY = CfCfg<In>::s2_every;
    __shared__ float4 lds[(YL ? CF_LDS4 + YLDS / 2 : CF_LDS4) + 12];
    float4 *xin = lds;
    float2 *lin = reinterpret_cast<float2 *>(lds + XIN4);
    float *yb = reinterpret_cast<float *>(lds + CF_LDS4);   // YL only: y as (re, im) floats
    // the 48 stage-1 taps in LDS, read as broadcast float4s beside the samples: as scalar operands
    // hipcc re-loads them every tile (SGPR pressure), and those scalar loads share lgkmcnt with the
    // LDS reads, so each sample read was waited for right before its use (one or two in flight)
    float4 *htap = lds + (YL ? CF_LDS4 + YLDS / 2 : CF_LDS4);
    if (threadIdx.x < 12)
        htap[threadIdx.x] = make_float4(h1[4 * threadIdx.x], h1[4 * threadIdx.x + 1], h1[4 * threadIdx.x + 2],
                                        h1[4 * threadIdx.x + 3]);
    const int ch = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const In *xp = iq + (size_t)ch * (ld / 2);   // N, ld even: 2 complex samples per load; rows ld apart
    float2 *yp = y + (size_t)ch * M2;           // (YL && FUSE: unused)
    int ybase = 0;   // y index of yb[0]
    // Stage-2 outputs collect in yb and go out in one coalesced burst when the channel is done (or
    // when YLDS fills): stores interleaved with the input stream cost ~0.3 ms per 8192-channel
    // batch at two workgroups per CU (HBM read/write turnarounds, and store acks inside the
    // prefetch's in-order vmcnt).
    auto flush = [&](int mend) {
        for (int i = tid; i < mend - ybase; i += 256) yp[ybase + i] = make_float2(yb[2 * i], yb[2 * i + 1]);
        ybase = mend;
    };
    float at[S2K];   // this lane's A fragments
#pragma unroll
    for (int k = 0; k < S2K; ++k) at[k] = afrag[64 * k + lane];
    // stage 2 reads whole windows, zero taps included: every entry must be finite
    for (int i = tid; i < LR; i += 256) lin[i] = make_float2(0.f, 0.f);
    int kbase = 0;   // x240 index of lin[0]
    // register prefetch PFD tiles deep (40 KiB in flight per workgroup): tile t's samples
    // [2560 t, 2560 t + 2560) land at image sample HALO + i
    // Loads are unconditional (index clamped) so the wait before a tile's LDS write can leave the
    // next tile's loads in flight.  Clamped samples past the end only feed stage-1 outputs k >= M1,
    // which are never computed (10 (M1-1) + 47 <= N-1).
    const long nq = N / 2;
    auto load_tile = [&](In (&pf)[5], int t) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            const long q = (long)t * (TILE_IN / 2) + r * 256 + tid;   // sample-pair index
            pf[r] = ld_nt(xp + min(q, nq - 1));   // streamed once: nt (common.h)
        }
    };
    int u_done = 0;   // stage-2 output triples [0, u_done) are stored
    auto tile = [&](int t, In (&pf)[5]) __attribute__((always_inline)) {
        const int kfirst = TILE_K * t - 4;   // stage-1 output of thread 0 in this tile
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            const float4 v = pair_f32(pf[r]);
            xin[HALO / 2 + r * 256 + tid] = make_float4(v.x, v.y, v.z, v.w);
        }
        // keep the re-load after the LDS writes so pf's registers are reused in place (otherwise
        // the scheduler hoists it and the loop latch copies registers under a full vmcnt(0))
        __builtin_amdgcn_sched_barrier(0);
        load_tile(pf, t + PFD);   // tile t+PFD in flight during compute (t+1.. already are)
        __syncthreads();
        // stage 1: x240[k] = sum_j h1[j] * x[10k + j], k = kfirst + tid; x[10k + j] is sample
        // 10 tid + 8 + j of the image
        const int k = kfirst + tid;
        if (k >= 0 && k < M1) {
            const float4 *w = xin + 5 * tid + 4;
            pf2 a = {0.f, 0.f};
            if constexpr (YL) {   // three groups of 16 taps, the next group's reads in flight
                float4 ta[4], xa[8], tb[4], xb[8];
                auto rd = [&](float4 (&T)[4], float4 (&X)[8], int g) __attribute__((always_inline)) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        T[i] = htap[4 * g + i];
                        X[2 * i] = w[8 * g + 2 * i];
                        X[2 * i + 1] = w[8 * g + 2 * i + 1];
                    }
                };
                auto fm = [&](const float4 (&T)[4], const float4 (&X)[8]) __attribute__((always_inline)) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float4 t4 = T[i], x0 = X[2 * i], x1 = X[2 * i + 1];
                        a = pfma(t4.x, pf2{x0.x, x0.y}, a);
                        a = pfma(t4.y, pf2{x0.z, x0.w}, a);
                        a = pfma(t4.z, pf2{x1.x, x1.y}, a);
                        a = pfma(t4.w, pf2{x1.z, x1.w}, a);
                    }
                };
                rd(ta, xa, 0);
                rd(tb, xb, 1);
                __builtin_amdgcn_sched_barrier(0);
                fm(ta, xa);
                __builtin_amdgcn_sched_barrier(0);
                rd(ta, xa, 2);
                __builtin_amdgcn_sched_barrier(0);
                fm(tb, xb);
                __builtin_amdgcn_sched_barrier(0);
                fm(ta, xa);
            } else {   // SC16 keeps the scalar taps (VGPR budget, below; LDS taps read two quads ahead
                       // of the chain measured 3 % slower: 1.20 -> 1.24 ms per pipelined SC16 step)
#pragma unroll
                for (int jj = 0; jj < 24; ++jj) {
                    const float4 v = w[jj];
                    a = pfma(h1[2 * jj], pf2{v.x, v.y}, a);
                    a = pfma(h1[2 * jj + 1], pf2{v.z, v.w}, a);
                }
            }
            lin[k - kbase] = make_float2(a.x, a.y);
        }
        __syncthreads();
        // halo for the next tile: image samples [0, 48) = this tile's [2560, 2608)
        if (tid < HALO / 2) xin[tid] = xin[TILE_IN / 2 + tid];
        const int kav = min(kfirst + TILE_K - 1, M1 - 1);   // last stage-1 output available
        const bool last = kav == M1 - 1;
        if (t % S2_EVERY == S2_EVERY - 1 || last) {
            // stage 2: triples u whose three outputs have all taps available (all of them at the end)
            const int num = 3 * kav + 2 - 320;   // largest m with floor((320 + 10m)/3) <= kav
            const int m_hi = num >= 0 ? min(num / 10, M2 - 1) : -1;
            const int u_hi = last ? (M2 - 1) / 3 : (m_hi >= 2 ? (m_hi - 2) / 3 : -1);
            const int nt = u_hi >= u_done ? (u_hi - u_done + S2T) / S2T : 0;   // MFMA tiles
            const int mend = min(3 * (u_hi + 1), M2);
            if (YL && nt > 0 && mend - ybase > YLDS) {   // this burst would not fit
                flush(3 * u_done);
                __syncthreads();
            }
            // columns: lane & 15 = 2 seg + comp; k-group lane >> 4.  Tile pairs (2p, 2p + 1) go to
            // wave p % 4: two independent accumulators per wave cover the MFMA's latency.
            const int kg = lane >> 4, seg = (lane & 15) >> 1, comp = lane & 1;
            const float *lf = reinterpret_cast<const float *>(lin);
            float *ys = YL ? yb : reinterpret_cast<float *>(xin + HALO / 2);   // !YL: staged, stored below
            const int yo = YL ? ybase : 3 * u_done;
            for (int p = wv; 2 * p < nt; p += 4) {
                const int U0 = u_done + 2 * p * S2T + S2Q * seg, U1 = U0 + S2T;
                // a column past u_hi reads the buffer's start instead (finite, never stored)
                const int b0 = U0 <= u_hi ? 2 * (10 * U0 - kbase + kg) + comp : 2 * kg + comp;
                const int b1 = U1 <= u_hi ? 2 * (10 * U1 - kbase + kg) + comp : 2 * kg + comp;
                f4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
                if constexpr (YL) {
                    // B operands a third of the chain ahead (hipcc otherwise waits lgkmcnt(0), one
                    // LDS round trip, before each MFMA pair).  Not for SC16: the 26 extra VGPRs
                    // take it from 120 to 161, four workgroups per CU to three (1.10 -> 1.57 ms)
                    float bv0[S2K], bv1[S2K];
#pragma unroll
                    for (int s3 = 0; s3 < 3; ++s3) {
#pragma unroll
                        for (int s2 = 13 * s3; s2 < 13 * s3 + 13; ++s2) {
                            bv0[s2] = lf[b0 + 8 * s2];
                            bv1[s2] = lf[b1 + 8 * s2];
                        }
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int s2 = 13 * s3; s2 < 13 * s3 + 13; ++s2) {
                            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(at[s2], bv0[s2], c0, 0, 0, 0);
                            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(at[s2], bv1[s2], c1, 0, 0, 0);
                        }
                    }
                } else {
#pragma unroll
                    for (int s2 = 0; s2 < S2K; ++s2) {
                        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(at[s2], lf[b0 + 8 * s2], c0, 0, 0, 0);
                        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(at[s2], lf[b1 + 8 * s2], c1, 0, 0, 0);
                    }
                }
                // D: this lane holds rows i = 4 kg + r of its column; output m = 3 U + i
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 4 * kg + r, q = i / 3;
                    if (i < 15) {
                        const int m0 = 3 * U0 + i, m1 = 3 * U1 + i;
                        if (U0 + q <= u_hi && m0 < M2) ys[2 * (m0 - yo) + comp] = c0[r];
                        if (U1 + q <= u_hi && m1 < M2) ys[2 * (m1 - yo) + comp] = c1[r];
                    }
                }
            }
            if constexpr (!YL) {
                if (nt > 0) {   // coalesced store of this burst's outputs y[3 u_done, mend)
                    __syncthreads();
                    // sc1 (copy_out): 1.11 -> 1.09 ms per SC16 batch, same box
                    copy_out(reinterpret_cast<uint8_t *>(yp + yo), reinterpret_cast<const uint8_t *>(ys), 8 * (mend - yo), tid);
                }
            }
            if (u_hi + 1 > u_done) u_done = u_hi + 1;
            if (!last) {
                // keep x240[10 u_done, kav] (the next triples' windows) at the buffer's front
                const int from = 10 * u_done - kbase, cnt = kav + 1 - 10 * u_done;
                __syncthreads();
                const float2 v = tid < cnt ? lin[from + tid] : make_float2(0.f, 0.f);
                __syncthreads();
                if (tid < cnt) lin[tid] = v;
                kbase = 10 * u_done;
            }
        }
        __syncthreads();
    };
    const int ntile = (M1 + 4 + TILE_K - 1) / TILE_K;   // tiles with kfirst < M1
    // two register sets, explicitly (a pr[PFD][5] array with unrolled loops over it cost 22-30 VGPRs:
    // SC16 at 142 instead of 120 lost its fourth workgroup per CU)
    static_assert(PFD == 2, "pa / pb below");
    In pa[5], pb[5];
    load_tile(pa, 0);
    load_tile(pb, 1);
    int t = 0;
    for (; t + 1 < ntile; t += 2) {
        tile(t, pa);
        tile(t + 1, pb);
    }
    if (t < ntile) tile(t, pa);
    // the last tile ended with a barrier
    if constexpr (FUSE) {
        const float2 *ly = reinterpret_cast<const float2 *>(yb);   // YL: yb holds y[0, M2)
        float2 *scr = reinterpret_cast<float2 *>(xin);
        if constexpr (!YL) {
            // y (this workgroup's stores) back into LDS, the timing scratch after it (the launch
            // guarantees M2 + smax <= CF_LDS2_SC16).  Workgroup-scope fence: the stores and the loads
            // share this CU's L1 (a device-scope fence would write back the whole L2 per channel).
            __threadfence_block();
            __syncthreads();
            float2 *yl = reinterpret_cast<float2 *>(lds);
            for (int i0 = tid; i0 < M2; i0 += 4 * 256) {
                float2 v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = i0 + 256 * e < M2 ? yp[i0 + 256 * e] : make_float2(0.f, 0.f);
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (i0 + 256 * e < M2) yl[i0 + 256 * e] = v[e];
            }
            __syncthreads();
            ly = yl;
            scr = yl + M2;
        }
        __shared__ TrackOut tro;
        __shared__ int prog;
        timing_tail(ly, scr, to, M2, ch, tid, &tro, &prog);
    } else if constexpr (YL) {
        flush(M2);
    }
}

// --------------------------------------------------------------------------- per-wave channel filter
// cf32 and SC16 with y in LDS (M2 <= YLDS): the workgroup's waves stream the channel's quarters
// independently.  Wave w owns the stage-2 triples [U_w, U_w+1) and the stage-1 outputs
// [K_w, K_w+1), K_w = 10 U_w (the last wave's end is M1), in wave tiles with its own LDS image and
// stage-1 buffer, and runs a one-MFMA-tile stage-2 burst (40 triples: one dependent chain of 39
// MFMAs) whenever 40 triples have their windows.  So the stream has no workgroup barrier until the
// channel ends, and a burst stalls one wave's quarter of the loads in flight instead of the whole
// workgroup's (k_chanfilt: every wave waits at the tile's barriers while three of them run the
// burst's MFMA pairs).  Wave w's last triples need stage-1 outputs up to K_w+1 + 103, the first
// ones of wave w + 1, which that wave also copies into a seam buffer.  A wave bursts every ready
// triple at its last tile, so after the one barrier at the channel's end it appends its seam and
// runs one burst of the <= 12 triples left, then the timing tail as in k_chanfilt.  Every output is
// the same fma chain as in k_chanfilt (bit-identical to the oracle).  (Round 3 ran cf32 on
// k_chanfilt_w, the same structure with each lane reading its whole 48-sample window and the taps
// from LDS; k_chanfilt_r below replaced it)
constexpr int WLR = 568;                    // wave stage-1 buffer (float2): < 567 entries in the stream,
                                            // <= 265 in the channel's last (seam) burst
constexpr int SEAM = 112;                   // >= the 104 outputs a left neighbour's last triples need
constexpr int UMIN = 16;                    // triples per wave at least (10 UMIN >= SEAM)
static_assert(sizeof(TrackOut) + sizeof(int) <= 48 && (4 * WLR + 3 * SEAM) % 2 == 0, "per-wave demod LDS carving");
constexpr int WTAIL_SM = YLDS / 4 + 3;      // the fused tail's symbols per channel at most (+1: a continued
                                            // stream's carried symbol 0)

// cross-lane LDS hand-off inside one wave: a wave's LDS instructions execute in order, so only the
// compiler has to be kept from moving accesses across this point (no s_waitcnt, no s_barrier)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// --------------------------------------------------------------------------- register stage 1
// k_chanfilt_r: the per-wave channel filter with stage 1 out of LDS.  With each lane reading its
// whole 48-sample window (24 float4) and the 48 taps (12 broadcast float4) from LDS for one output
// (round 3's k_chanfilt_w), stage 1 costs ~5 LDS cycles per output of the CU's 128 B/cycle, and
// that bounds the filter once the input needs no HBM (timing builds, input L2-resident: 0.93 ms per
// 8192 x 131072 batch without the tail; with stage 1's chain cut to a third, 0.66).  Here a lane reads
// only its own 10-sample block from the image (5 loads of 2 samples) and takes the next four blocks
// from its row neighbours with DPP (row_shl:p reads lane + p of the same 16-lane row): a row of 16
// lanes holds 16 consecutive blocks and computes the outputs of its first 12, so a wave tile is 48
// outputs (480 new samples, a 40-sample halo).  The taps sit in registers.  Each output is still the
// oracle's ascending-j fma chain (x[10 k + j] is sample j mod 10 of lane + j / 10's block),
// bit-identical.  SC16 keeps its samples as raw dwords in the image (re low 16 bits, im high) and
// folds the 2^-15 scale into the taps (an exact power of two: fma(h 2^-15, x, a) == fma(h, x 2^-15, a)).
constexpr int RHALO = 40;           // image samples carried over from the previous tile
template <typename In> struct RCfg;
// nb: 10-sample blocks per lane.  nb = 1: a row's 16 lanes hold 16 blocks and compute the outputs
// of the first 12 (DPP shifts of 1..4 lanes); nb = 2: lane i holds blocks 2i, 2i + 1, a row 32
// blocks, outputs of the first 28 (shifts of 1..2 lanes) -- 14 of 16 lanes' work kept instead of 12
// and the per-tile work (loads, image, halo, burst test) spread over 112 outputs instead of 48.
// cf32 keeps nb = 1: its 9.3 KB nb = 2 image would not fit two workgroups per CU.
// pf: input tiles in flight per wave (register prefetch).
template <> struct RCfg<uint4> { static constexpr int bps = 4, pf = 2, nb = 2, wlr = 632; };   // SC16: 16-B load = 4 samples
template <> struct RCfg<float4> { static constexpr int bps = 8, pf = 3, nb = 1, wlr = WLR; };  // cf32: 2 samples (4 tiles: spills)
template <typename In> constexpr int r_tk() { return RCfg<In>::nb == 1 ? 48 : 112; }   // stage-1 outputs per wave tile
template <typename In> constexpr int r_chunks() { return 10 * r_tk<In>() * RCfg<In>::bps / 16; }   // 16-B loads per tile
// per-wave image: two halo slots (tile t reads slot t & 1; tile t's last RHALO samples are also
// written into slot (t + 1) & 1 as they arrive, so no halo copy) + the tile's 10 TK samples
template <typename In> constexpr int r_img16() { return (2 * RHALO + 10 * r_tk<In>()) * RCfg<In>::bps / 16; }
template <typename In> constexpr int r_smem4() {
    return 3 + 4 * r_img16<In>() + (4 * RCfg<In>::wlr + 3 * SEAM + YLDS) / 2;
}
// tail staging over the freed images + stage-1 buffers: d_j, soft bits, hard dibits, O-M parts, symbols
constexpr int r_tail_bytes() { return 19 * WTAIL_SM + 48 + 1024; }
static_assert(r_tail_bytes() <= 4 * r_img16<float4>() * 16 + 4 * WLR * 8, "k_chanfilt_r tail staging");
// two workgroups per CU with >= 9.5 KB of the CU's LDS left for the lower MAC's kernels
// (k_etsi_viterbi 7 KB, k_etsi_sync 2.4 KB), which the bench's pipeline runs beside the next demod
static_assert(2 * r_smem4<float4>() * 16 + 7 * 1024 + 2560 <= 160 * 1024, "k_chanfilt_r LDS (cf32)");
static_assert(2 * r_smem4<uint4>() * 16 + 7 * 1024 + 2560 <= 160 * 1024, "k_chanfilt_r LDS (SC16)");
// a stage-1 buffer holds < 10 x 39 + 123 + one tile's outputs (the burst test runs once per tile)
static_assert(RCfg<uint4>::wlr >= 513 + 112 && WLR >= 513 + 48, "stage-1 buffer");

// ar += h[q] * x_re[q], ai += h[q] * x_im[q] for q < N in order, x taken from lane + P of this
// lane's 16-lane row (row_shl:P; a lane past the row's end reads 0 -- only lanes whose outputs are
// not kept do): one v_fmac_f32_dpp per product, the DPP folded into the fma (hipcc emits a
// v_mov_b32_dpp per operand instead and keeps ~76 of them live).  Five products per asm: the hazard
// recognizer puts a wait state after every asm statement.  A DPP read needs two wait states after
// the VALU write of its source: where the chain's order does not already put this lane's own use
// of x (and so its conversion) >= 9 steps earlier, NOP = true opens the block with s_nop 1.
template <int P, int N, bool NOP = false>
__device__ __forceinline__ void fmac_rows(float &ar, float &ai, const float *xr, const float *xi, const float *h) {
    if constexpr (P == 0) {   // in-lane: one v_pk_fma_f32 per product (both halves' fma, the same bits)
        pf2 a = {ar, ai};
#pragma unroll
        for (int q = 0; q < N; ++q) a = pfma(h[q], pf2{xr[q], xi[q]}, a);
        ar = a.x;
        ai = a.y;
    }
    else if constexpr (P == 1 && N == 5 && !NOP) {
        asm("v_fmac_f32_dpp %0, %2, %12 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %12 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %13 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %8, %13 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %14 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %9, %14 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %5, %15 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %10, %15 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %6, %16 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %11, %16 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xr[3]), "v"(xr[4]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(xi[3]), "v"(xi[4]), "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]), "v"(h[4]));
    }
    else if constexpr (P == 1 && N == 5 && NOP) {
        asm("s_nop 1\n\t"
            "v_fmac_f32_dpp %0, %2, %12 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %12 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %13 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %8, %13 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %14 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %9, %14 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %5, %15 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %10, %15 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %6, %16 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %11, %16 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xr[3]), "v"(xr[4]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(xi[3]), "v"(xi[4]), "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]), "v"(h[4]));
    }
    else if constexpr (P == 1 && N == 3 && !NOP) {
        asm("v_fmac_f32_dpp %0, %2, %8 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %5, %8 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %6, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %10 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %10 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(h[0]), "v"(h[1]), "v"(h[2]));
    }
    else if constexpr (P == 1 && N == 3 && NOP) {
        asm("s_nop 1\n\t"
            "v_fmac_f32_dpp %0, %2, %8 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %5, %8 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %6, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %10 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %10 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(h[0]), "v"(h[1]), "v"(h[2]));
    }
    else if constexpr (P == 2 && N == 5 && !NOP) {
        asm("v_fmac_f32_dpp %0, %2, %12 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %12 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %13 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %8, %13 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %14 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %9, %14 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %5, %15 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %10, %15 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %6, %16 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %11, %16 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xr[3]), "v"(xr[4]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(xi[3]), "v"(xi[4]), "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]), "v"(h[4]));
    }
    else if constexpr (P == 2 && N == 5 && NOP) {
        asm("s_nop 1\n\t"
            "v_fmac_f32_dpp %0, %2, %12 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %12 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %13 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %8, %13 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %14 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %9, %14 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %5, %15 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %10, %15 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %6, %16 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %11, %16 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xr[3]), "v"(xr[4]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(xi[3]), "v"(xi[4]), "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]), "v"(h[4]));
    }
    else if constexpr (P == 2 && N == 3 && !NOP) {
        asm("v_fmac_f32_dpp %0, %2, %8 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %5, %8 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %9 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %6, %9 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %10 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %10 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(h[0]), "v"(h[1]), "v"(h[2]));
    }
    else if constexpr (P == 2 && N == 3 && NOP) {
        asm("s_nop 1\n\t"
            "v_fmac_f32_dpp %0, %2, %8 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %5, %8 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %9 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %6, %9 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %10 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %10 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(h[0]), "v"(h[1]), "v"(h[2]));
    }
    else if constexpr (P == 3 && N == 5 && !NOP) {
        asm("v_fmac_f32_dpp %0, %2, %12 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %12 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %13 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %8, %13 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %14 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %9, %14 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %5, %15 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %10, %15 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %6, %16 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %11, %16 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xr[3]), "v"(xr[4]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(xi[3]), "v"(xi[4]), "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]), "v"(h[4]));
    }
    else if constexpr (P == 3 && N == 5 && NOP) {
        asm("s_nop 1\n\t"
            "v_fmac_f32_dpp %0, %2, %12 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %12 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %13 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %8, %13 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %14 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %9, %14 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %5, %15 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %10, %15 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %6, %16 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %11, %16 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xr[3]), "v"(xr[4]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(xi[3]), "v"(xi[4]), "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]), "v"(h[4]));
    }
    else if constexpr (P == 3 && N == 3 && !NOP) {
        asm("v_fmac_f32_dpp %0, %2, %8 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %5, %8 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %9 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %6, %9 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %10 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %10 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(h[0]), "v"(h[1]), "v"(h[2]));
    }
    else if constexpr (P == 3 && N == 3 && NOP) {
        asm("s_nop 1\n\t"
            "v_fmac_f32_dpp %0, %2, %8 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %5, %8 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %9 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %6, %9 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %10 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %10 row_shl:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(h[0]), "v"(h[1]), "v"(h[2]));
    }
    else if constexpr (P == 4 && N == 5 && !NOP) {
        asm("v_fmac_f32_dpp %0, %2, %12 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %12 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %13 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %8, %13 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %14 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %9, %14 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %5, %15 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %10, %15 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %6, %16 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %11, %16 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xr[3]), "v"(xr[4]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(xi[3]), "v"(xi[4]), "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]), "v"(h[4]));
    }
    else if constexpr (P == 4 && N == 5 && NOP) {
        asm("s_nop 1\n\t"
            "v_fmac_f32_dpp %0, %2, %12 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %12 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %13 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %8, %13 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %14 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %9, %14 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %5, %15 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %10, %15 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %6, %16 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %11, %16 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xr[3]), "v"(xr[4]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(xi[3]), "v"(xi[4]), "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]), "v"(h[4]));
    }
    else if constexpr (P == 4 && N == 3 && !NOP) {
        asm("v_fmac_f32_dpp %0, %2, %8 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %5, %8 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %9 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %6, %9 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %10 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %10 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(h[0]), "v"(h[1]), "v"(h[2]));
    }
    else if constexpr (P == 4 && N == 3 && NOP) {
        asm("s_nop 1\n\t"
            "v_fmac_f32_dpp %0, %2, %8 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %5, %8 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %3, %9 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %6, %9 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %0, %4, %10 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f32_dpp %1, %7, %10 row_shl:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            : "+v"(ar), "+v"(ai)
            : "v"(xr[0]), "v"(xr[1]), "v"(xr[2]), "v"(xi[0]), "v"(xi[1]), "v"(xi[2]), "v"(h[0]), "v"(h[1]), "v"(h[2]));
    }
    else {
        static_assert(P == 0, "fmac_rows: no such form");
    }
}

// (Round 4 measured and removed a form with y in a global scratch, one tile prefetched and three
// workgroups per CU for SC16: 0.938 -> 1.05 ms)
template <typename In, bool FUSE>
__global__ __launch_bounds__(256, 2) void k_chanfilt_r(const In *__restrict__ iq, long N, int M1, int M2,
                                                       const float *__restrict__ h1, const float *__restrict__ afrag,
                                                       float2 *__restrict__ y, TimingOut to, long ld) {
    constexpr bool SC16 = std::is_same<In, uint4>::value;
    constexpr int BPS = RCfg<In>::bps, PF = RCfg<In>::pf, NCH = r_chunks<In>(), NL = (NCH + 63) / 64;
    constexpr int NB = RCfg<In>::nb, TK = r_tk<In>(), TIN = 10 * TK, LR = RCfg<In>::wlr;
    constexpr int ROWK = NB == 1 ? 12 : 28;    // outputs per 16-lane row
    constexpr int RH16 = RHALO * BPS / 16;     // 16-B chunks per halo
    constexpr int IMGB = r_img16<In>() * 16;   // image bytes per wave
    using Pair = typename std::conditional<SC16, uint2, float4>::type;   // two samples
    __shared__ float4 smem[r_smem4<In>()];
    TrackOut *tro = reinterpret_cast<TrackOut *>(smem);                        // + prog: 3 float4
    uint8_t *img_all = reinterpret_cast<uint8_t *>(smem + 3);                  // 4 wave images
    float2 *lin_all = reinterpret_cast<float2 *>(img_all + 4 * IMGB);          // 4 stage-1 buffers
    float2 *seam = lin_all + 4 * LR;
    const int ch = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const uint32_t t_start = FUSE && to.probe && tid == 0 ? (uint32_t)wall_clock64() : 0u;
    float *yb = reinterpret_cast<float *>(seam + 3 * SEAM);
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint8_t *img = img_all + wv * IMGB;
    float2 *lin = lin_all + wv * LR;
    for (int i = lane; i < LR; i += 64) lin[i] = make_float2(0.f, 0.f);
    float at[S2K];
#pragma unroll
    for (int k = 0; k < S2K; ++k) at[k] = afrag[64 * k + lane];
    // SC16: the launch passes the taps pre-scaled by 2^-15.  Taps 10..47 are v_fmac_f32_dpp's src1 and
    // must be VGPRs (left as SGPRs hipcc copies them into VGPRs every tile); taps 0..9 (the in-lane
    // products) stay scalar operands
    float hv[48];
#pragma unroll
    for (int j = 0; j < 48; ++j) {
        hv[j] = h1[j];
        if (j >= 10) asm volatile("" : "+v"(hv[j]));
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): landed before the stream starts
    // the partition
    const int UT = (M2 + 2) / 3;
    const int nw = min(4, max(1, UT / UMIN));
    const int UQ = (UT + nw - 1) / nw;
    const bool active = wv < nw;
    const bool has_right = wv + 1 < nw;
    const int u_beg = min(wv * UQ, UT), u_end = has_right ? (wv + 1) * UQ : UT;
    const int K0 = 10 * u_beg, K1 = has_right ? 10 * u_end : M1;
    const int ntile = active ? (K1 - K0 + 4 + TK - 1) / TK : 0;   // wave tiles with kfirst < K1
    // tile t: lane (row ro, i) holds the NB blocks of x240[K0 + TK t - 4 + ROWK ro + NB i + e], e < NB,
    // samples 10 (K0 + TK t) - 40 + 10 (ROWK ro + NB i + e) + [0, 10) = image samples
    // 10 (ROWK ro + NB i + e) + [0, 10); the tile's new samples 10 (K0 + TK t) + [0, 10 TK) land at
    // image sample 40.  A buffer resource over the wave's samples [10 K0, last needed]: loads past
    // it return 0 without touching memory.
    const long s0 = 10L * K0;
    const long slast = active ? min(10L * (K1 - 1) + 47, N - 1) : s0;
    const uint8_t *xp = reinterpret_cast<const uint8_t *>(iq) + ((size_t)ch * ld + s0) * BPS;   // rows ld apart
    const int nbytes = active ? (int)(((slast - s0 + 1) * BPS + 15) & ~15L) : 0;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(xp), 0, nbytes, 0x00020000);
    const int ro = lane >> 4, li = lane & 15;
    const int blk = ROWK * ro + NB * li;   // this lane's first block
    auto load_tile = [&](In (&pf)[NL], int t) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < NL; ++r) {
            const int c = min(64 * r + lane, NCH - 1);   // unconditional (a branch makes hipcc wait at the join)
            const nt_f4 v = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * c, t * TIN * BPS, 2 /* nt */);
            pf[r] = *reinterpret_cast<const In *>(&v);
        }
    };
    int kbase = K0;      // x240 index of lin[0]
    int u_done = u_beg;  // triples [u_beg, u_done) are in yb
    const int kg = lane >> 4, seg = (lane & 15) >> 1, comp = lane & 1;
    const float *lf = reinterpret_cast<const float *>(lin);
    // one MFMA tile: triples [u_done, u_done + 40) as 8 segments x 5 (columns = 2 seg + comp), only
    // triples < u_lim stored; a column past u_lim reads the buffer's start (finite, never stored).
    // B operands one 13-step chunk ahead of the MFMAs that use them (hipcc otherwise waits one LDS
    // round trip before every MFMA pair of the dependent chain)
    auto burst = [&](int u_lim) __attribute__((always_inline)) {
        const int U0 = u_done + S2Q * seg;
        const int b0 = U0 < u_lim ? 2 * (10 * U0 - kbase + kg) + comp : 2 * kg + comp;
        float bv[S2K];
        f4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 13; ++s2) bv[s2] = lf[b0 + 8 * s2];
#pragma unroll
        for (int s3 = 0; s3 < 3; ++s3) {
            __builtin_amdgcn_sched_barrier(0);
            if (s3 < 2) {
#pragma unroll
                for (int s2 = 13 * s3 + 13; s2 < 13 * s3 + 26; ++s2) bv[s2] = lf[b0 + 8 * s2];
            }
#pragma unroll
            for (int s2 = 13 * s3; s2 < 13 * s3 + 13; ++s2)
                c = __builtin_amdgcn_mfma_f32_16x16x4f32(at[s2], bv[s2], c, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 4 * kg + r, q = i / 3, m = 3 * U0 + i;
            if (i < 15 && U0 + q < u_lim && m < M2) yb[2 * m + comp] = c[r];
        }
    };
    auto tile = [&](int t, In (&pf)[NL]) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < NL; ++r)
            if (64 * r + lane < NCH) *reinterpret_cast<In *>(img + 2 * RHALO * BPS + 16 * (64 * r + lane)) = pf[r];
        // the tile's last RHALO samples: also the next tile's halo slot
#pragma unroll
        for (int r = 0; r < NL; ++r) {
            const int c = 64 * r + lane - (NCH - RH16);
            if (c >= 0 && c < RH16) *reinterpret_cast<In *>(img + ((t + 1) & 1) * RHALO * BPS + 16 * c) = pf[r];
        }
        __builtin_amdgcn_sched_barrier(0);
        load_tile(pf, t + PF);
        wave_sync();
        // this lane's blocks: 10 NB samples as 5 NB pairs; image sample s < RHALO is in halo slot
        // t & 1, the rest at 2 RHALO + (s - RHALO) (a lane's blocks lie on one side: blk < 4 or >= 4)
        const uint8_t *bimg = img + (10 * blk + (blk < 4 ? (t & 1) * RHALO : RHALO)) * BPS;
        float xre[10 * NB], xim[10 * NB];
#pragma unroll
        for (int m = 0; m < 5 * NB; ++m) {
            const Pair v = *reinterpret_cast<const Pair *>(bimg + 2 * m * BPS);
            if constexpr (SC16) {
                xre[2 * m] = (float)(int16_t)(v.x & 0xFFFFu);
                xim[2 * m] = (float)(int16_t)(v.x >> 16);
                xre[2 * m + 1] = (float)(int16_t)(v.y & 0xFFFFu);
                xim[2 * m + 1] = (float)(int16_t)(v.y >> 16);
            } else {
                xre[2 * m] = v.x;
                xim[2 * m] = v.y;
                xre[2 * m + 1] = v.z;
                xim[2 * m + 1] = v.w;
            }
        }
        // x240[k] = sum_j h1[j] x[10 k + j], j ascending: sample j % 10 of block k + j / 10
        const int k = K0 + TK * t - 4 + blk;
        if constexpr (NB == 1) {   // block k + p: lane + p
            float ar = 0.f, ai = 0.f;
            fmac_rows<0, 10>(ar, ai, xre, xim, hv);
            fmac_rows<1, 5>(ar, ai, xre, xim, hv + 10);
            fmac_rows<1, 5>(ar, ai, xre + 5, xim + 5, hv + 15);
            fmac_rows<2, 5>(ar, ai, xre, xim, hv + 20);
            fmac_rows<2, 5>(ar, ai, xre + 5, xim + 5, hv + 25);
            fmac_rows<3, 5>(ar, ai, xre, xim, hv + 30);
            fmac_rows<3, 5>(ar, ai, xre + 5, xim + 5, hv + 35);
            fmac_rows<4, 5>(ar, ai, xre, xim, hv + 40);
            fmac_rows<4, 3>(ar, ai, xre + 5, xim + 5, hv + 45);
            if (li < 12 && k >= K0 && k < K1) {
                lin[k - kbase] = make_float2(ar, ai);
                if (wv > 0 && k - K0 < SEAM) seam[(wv - 1) * SEAM + k - K0] = make_float2(ar, ai);
            }
        } else {   // output A = block k: blocks k, k+1 in-lane, k+2, k+3 lane + 1, k+4 lane + 2;
                   // output B = block k + 1: k+1 in-lane, k+2, k+3 lane + 1, k+4, k+5 lane + 2
            const float *x0r = xre, *x0i = xim, *x1r = xre + 10, *x1i = xim + 10;
            float ar = 0.f, ai = 0.f, br = 0.f, bi = 0.f;
            fmac_rows<0, 10>(ar, ai, x0r, x0i, hv);
            fmac_rows<0, 10>(ar, ai, x1r, x1i, hv + 10);
            fmac_rows<0, 10>(br, bi, x1r, x1i, hv);
            fmac_rows<1, 5, true>(br, bi, x0r, x0i, hv + 10);   // x0's first read in B's chain
            fmac_rows<1, 5>(ar, ai, x0r, x0i, hv + 20);
            fmac_rows<1, 5, true>(br, bi, x0r + 5, x0i + 5, hv + 15);   // and of x0[5..9]
            fmac_rows<1, 5>(ar, ai, x0r + 5, x0i + 5, hv + 25);
            fmac_rows<1, 5>(br, bi, x1r, x1i, hv + 20);
            fmac_rows<1, 5>(ar, ai, x1r, x1i, hv + 30);
            fmac_rows<1, 5>(br, bi, x1r + 5, x1i + 5, hv + 25);
            fmac_rows<1, 5>(ar, ai, x1r + 5, x1i + 5, hv + 35);
            fmac_rows<2, 5>(br, bi, x0r, x0i, hv + 30);
            fmac_rows<2, 5>(ar, ai, x0r, x0i, hv + 40);
            fmac_rows<2, 5>(br, bi, x0r + 5, x0i + 5, hv + 35);
            fmac_rows<2, 3>(ar, ai, x0r + 5, x0i + 5, hv + 45);
            fmac_rows<2, 5>(br, bi, x1r, x1i, hv + 40);
            fmac_rows<2, 3>(br, bi, x1r + 5, x1i + 5, hv + 45);
            if (li < 14) {
                const bool va = k >= K0 && k < K1, vb = k + 1 >= K0 && k + 1 < K1;
                if (va && vb) {   // the two outputs side by side: one 16-B store
                    *reinterpret_cast<float4 *>(lin + (k - kbase)) = make_float4(ar, ai, br, bi);
                } else {
                    if (va) lin[k - kbase] = make_float2(ar, ai);
                    if (vb) lin[k + 1 - kbase] = make_float2(br, bi);
                }
                if (wv > 0) {
                    if (va && k - K0 < SEAM) seam[(wv - 1) * SEAM + k - K0] = make_float2(ar, ai);
                    if (vb && k + 1 - K0 < SEAM) seam[(wv - 1) * SEAM + k + 1 - K0] = make_float2(br, bi);
                }
            }
        }
        wave_sync();
        const int kav = min(K0 + TK * t + TK - 5, K1 - 1);   // the tile's last output
        const int u_rdy = kav >= 113 ? min((kav - 113) / 10 + 1, u_end) : 0;
        while (u_rdy - u_done >= S2T || (t == ntile - 1 && u_rdy > u_done)) {
            const int ul = min(u_done + S2T, u_rdy);
            burst(ul);
            u_done = ul;
            // keep x240[10 u_done, kav] at the buffer's front: <= 10 (one tile's triples) + 123
            const int from = 10 * u_done - kbase, cnt = kav + 1 - 10 * u_done;
            constexpr int NE = (TK + 123 + 63) / 64;
            float2 v[NE];
#pragma unroll
            for (int e = 0; e < NE; ++e) v[e] = lane + 64 * e < cnt ? lin[from + lane + 64 * e] : make_float2(0.f, 0.f);
            wave_sync();
#pragma unroll
            for (int e = 0; e < NE; ++e)
                if (lane + 64 * e < cnt) lin[lane + 64 * e] = v[e];
            kbase = 10 * u_done;
        }
        wave_sync();
    };
    In pf[PF][NL];
    if (ntile > 0) {
#pragma unroll
        for (int u = 0; u < PF; ++u) load_tile(pf[u], u);
    }
    int t = 0;
    for (; t + PF <= ntile; t += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) tile(t + u, pf[u]);
    }
#pragma unroll
    for (int u = 0; u < PF - 1; ++u)
        if (t + u < ntile) tile(t + u, pf[u]);
    __syncthreads();   // every wave's seam and in-loop bursts
    if (active && u_done < u_end) {
        if (has_right) {
            for (int i = lane; i < SEAM; i += 64) lin[K1 - kbase + i] = seam[wv * SEAM + i];
            wave_sync();
        }
        burst(u_end);
    }
    __syncthreads();
    if constexpr (FUSE) {
        // the tail's LDS over the freed images and stage-1 buffers (the launch guarantees
        // sm <= WTAIL_SM): d_j scratch, soft bits, hard dibits, the O-M parts, then the symbols
        const int sm = M2 / 4 + 2;
        uint8_t *R = img_all;
        const int o_sb = (8 * sm + 15) & ~15, o_hd = o_sb + ((2 * sm + 15) & ~15), o_om = o_hd + ((sm + 15) & ~15);
        const TailStage st{reinterpret_cast<float2 *>(R + o_om + 1024), reinterpret_cast<int8_t *>(R + o_sb), R + o_hd};
        int *prog = reinterpret_cast<int *>(tro + 1);
        timing_tail(reinterpret_cast<const float2 *>(yb), reinterpret_cast<float2 *>(R), to, M2, ch, tid, tro, prog,
                    &st, reinterpret_cast<float *>(R + o_om), t_start);
    } else {
        copy_out(reinterpret_cast<uint8_t *>(y + (size_t)ch * M2), reinterpret_cast<const uint8_t *>(yb), 8 * M2, tid);
    }
}

// --------------------------------------------------------------------------- E3/E4 lower MAC
// training/tail patterns (EN 300 392-2 §9.4.4.3), LSB-first words
__host__ __device__ constexpr uint64_t packb(const int *p, int n) {
    uint64_t w = 0;
    for (int j = 0; j < n; ++j) w |= (uint64_t)p[j] << j;
    return w;
}
constexpr int QB[22] = {1, 0, 1, 1, 0, 1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 0, 1, 0, 1, 1, 0, 1};
constexpr int NB[22] = {1, 1, 0, 1, 0, 0, 0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 0, 0};
constexpr int PB[22] = {0, 1, 1, 1, 1, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0, 1, 1, 1, 0, 0};
constexpr int YB[38] = {1, 1, 0, 0, 0, 0, 0, 1, 1, 0, 0, 1, 1, 1, 0, 0, 1, 1, 1,
                        0, 1, 0, 0, 1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 0, 0, 1, 1, 1};
constexpr uint64_t W_HEAD = packb(QB + 10, 12), W_TAIL = packb(QB, 10), W_N = packb(NB, 22), W_P = packb(PB, 22),
                   W_Y = packb(YB, 38);

// up to 32 stream bits from pos, from the 32-bit view of the words: one funnel shift
__device__ __forceinline__ uint32_t bits32_at(const uint32_t *w, int pos) {
    const int q = pos >> 5;
    return __builtin_amdgcn_alignbit(w[q + 1], w[q], (uint32_t)(pos & 31));
}
__device__ __forceinline__ int matches32(uint32_t v, uint32_t pat, int len) {
    return len - __popc((v ^ pat) & (len == 32 ? 0xFFFFFFFFu : ((1u << len) - 1)));
}
__device__ __forceinline__ int punct_index(int j1) {   // rate 2/3, t=3, P=(1,2,5); 1-based
    const int g = (j1 - 1) / 3;
    const int r = j1 - 3 * g;
    return 8 * g + (r == 1 ? 1 : r == 2 ? 2 : 5);
}

constexpr int LMAC_MAXBITS = 2 * 2048;

// CRC-16 register as a linear function of the bits (GF(2)): reg(L bits) = INIT[L] ^ XOR over
// 1-bits at distance d from the end of T[d].  Lets the serial traceback, which emits bits last
// to first, check the CRC on the fly instead of a second serial pass.
struct CrcTab {
    uint32_t t[288];   // dwords: read with wave-uniform scalar loads
    uint32_t init[289];
};
constexpr uint32_t crc_step(uint32_t r) { return ((r & 0x8000u) ? ((r << 1) ^ 0x1021u) : (r << 1)) & 0xFFFFu; }
constexpr CrcTab make_crc_tab() {
    CrcTab c{};
    uint32_t r = crc_step(0x8000u);
    for (int d = 0; d < 288; ++d) { c.t[d] = r; r = crc_step(r); }
    uint32_t s = 0xFFFFu;
    for (int L = 0; L <= 288; ++L) { c.init[L] = s; s = crc_step(s); }
    return c;
}
__constant__ CrcTab CRC_TAB = make_crc_tab();

// --------------------------------------------------------------------------- E3 burst sync
struct Job {
    int ch, slot, burst, blk, kind, off;
};

// Job regions, one per block kind, so every Viterbi wave runs a single trellis length:
// SCH/F [0, 8C), SCH/HD [8C, 24C), BSCH [24C, 32C) (<= 8 bursts per channel chunk).
__host__ __device__ inline size_t job_base(int kind, size_t C) { return kind == 0 ? 0 : kind == 1 ? 8 * C : 24 * C; }
__host__ __device__ inline size_t job_cap(int kind, size_t C) { return kind == 1 ? 16 * C : 8 * C; }

// One wave per channel: pack hard bits, greedy burst scan, then allocate this channel's coded
// blocks dense job indices in each kind's region (one atomic per kind per channel; outputs are
// indexed by (channel, slot), so results do not depend on the allocation order).
constexpr int SYNC_WAVES = 4;   // channels per workgroup: one job-counter atomic per workgroup

struct SyncLds {
    uint64_t words_all[SYNC_WAVES][LMAC_MAXBITS / 64 + 2];
    int bstart_all[SYNC_WAVES][ETSI_MAXB], bkind_all[SYNC_WAVES][ETSI_MAXB];
    int per_all[SYNC_WAVES][3];
    unsigned long long block_old;
};

// Streaming: the dibits (and their soft bits) the scan left unconsumed -- from row dibit td0, T of
// them -- go in front of column R of the next rows, and lead[c] to their first unexamined bit (one
// wave).  Into other rows straight from k_etsi_sync; into these rows (tinfo) by k_etsi_tail, after
// the trellis has read them.
__device__ __forceinline__ void tail_move(const uint8_t *hard, const int8_t *soft, int stride, int ch, int td0, int T,
                                          int ph, int R, uint8_t *nhard, int8_t *nsoft, int32_t *lead, int lane) {
    const uint8_t *hrow = hard + (size_t)ch * stride;
    const int8_t *srow = soft + (size_t)ch * 2 * stride;
    uint8_t hv[4];
    int8_t s0[4], s1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = lane + 64 * u;
        hv[u] = i < T ? hrow[td0 + i] : 0;
        s0[u] = i < T ? srow[2 * (td0 + i)] : 0;
        s1[u] = i < T ? srow[2 * (td0 + i) + 1] : 0;
    }
    __builtin_amdgcn_s_waitcnt(0);   // every read done before a write (the rows may be these rows)
    __builtin_amdgcn_wave_barrier();
    uint8_t *nh = nhard + (size_t)ch * stride;
    int8_t *ns = nsoft + (size_t)ch * 2 * stride;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = lane + 64 * u;
        if (i < T) {
            nh[R - T + i] = hv[u];
            ns[2 * (R - T + i)] = s0[u];
            ns[2 * (R - T + i) + 1] = s1[u];
        }
    }
    if (lane == 0) lead[ch] = 2 * (R - T) + ph;
}

// Streaming (lead != null, tetra_lmac_etsi_stream): row c holds the previous chunk's unconsumed
// dibits in front of column R and this chunk's from R; the scan starts at row bit lead[c] and
// afterwards the dibits from the first bit not examined move in front of column R of the next rows
// (nsoft / nhard), lead[c] pointing at their first bit -- oracle/etsi.py Stream.
__device__ __forceinline__ void sync_group(SyncLds &L, int grp, const uint8_t *__restrict__ hard,
                                           const int32_t *__restrict__ nsym, int smax, int32_t *__restrict__ nburst,
                                           int32_t *__restrict__ bursts, int32_t *__restrict__ nblock,
                                           unsigned long long *__restrict__ jcount, Job *__restrict__ jobs, int C,
                                           int32_t *lead, int R, int32_t *tinfo, const int8_t *soft, uint8_t *nhard,
                                           int8_t *nsoft) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ch = grp * SYNC_WAVES + wv;
    auto &words_all = L.words_all;
    auto &bstart_all = L.bstart_all;
    auto &bkind_all = L.bkind_all;
    auto &per_all = L.per_all;
    auto &block_old = L.block_old;
    uint64_t *words = words_all[wv];
    int *bstart = bstart_all[wv], *bkind = bkind_all[wv];
    const int S = ch < C ? nsym[ch] : 0;
    const int nd = S > 1 ? S - 1 : 0;
    int d0 = 0, cur0 = 0, nrow = nd;   // the scan's first dibit / bit, the row's dibits from d0
    if (lead) {
        const int b = ch < C ? min(max(lead[ch], 0), 2 * R) : 2 * R;
        d0 = b >> 1;
        cur0 = b & 1;
        nrow = R + nd - d0;
    }
    int nbits = 2 * nrow;
    if (nbits > LMAC_MAXBITS) nbits = LMAC_MAXBITS;
    const uint8_t *hp = hard + (size_t)ch * smax + d0;
    const int lim = smax - d0;   // the row's symbols from hp
    // pack hard bits with ballots: a word holds 32 dibit symbols (bit 2i = b1, 2i+1 = b2), so lane j
    // of the ballot contributes bit j of the word: component j & 1 of symbol j >> 1.  Two ballots per
    // 64 symbols and no bit interleave (interleaving two 32-bit ballots was ~80 scalar 64-bit ops per
    // word, on the CU's one scalar unit shared by all its waves)
    const int nsy = nbits / 2;
    // symbols loaded 8 steps (512 symbols) at a time, all before the first ballot: a load per step
    // in the dependent loop cost one memory latency per 64 symbols
    constexpr int PK = 8;
    const int sl = lane >> 1, comp = lane & 1;
    for (int s00 = 0; s00 < nsy + 64; s00 += 64 * PK) {
    uint32_t hA[PK], hB[PK];
#pragma unroll
    for (int u = 0; u < PK; ++u) {
        const int s = s00 + 64 * u + sl;
        hA[u] = hp[min(s, lim - 1)];   // unconditional (in the row): no branch join waits per load
        hB[u] = hp[min(s + 32, lim - 1)];
    }
#pragma unroll
    for (int u = 0; u < PK; ++u) {
        const int s0 = s00 + 64 * u;
        if (s0 >= nsy + 64) break;   // uniform
        const int s = s0 + sl;
        const uint32_t a = s < nsy ? (comp ? hA[u] : hA[u] >> 1) & 1u : 0u;
        const uint32_t b = s + 32 < nsy ? (comp ? hB[u] : hB[u] >> 1) & 1u : 0u;
        const uint64_t wa = __ballot(a), wb = __ballot(b);
        if (lane == 0 && s0 / 32 + 1 < LMAC_MAXBITS / 64 + 2) {
            words[s0 / 32] = wa;
            words[s0 / 32 + 1] = wb;
        }
    }
    }
    __syncthreads();
    int nb = 0;
    int nextpos = cur0;   // the first position not examined (streaming: where the next chunk resumes)
    for (int cur = cur0; cur + 510 <= nbits && nb < ETSI_MAXB;) {
        const int s = cur + lane;
        int kind = -1;
        if (s + 510 <= nbits) {
            // 32-bit funnel-shift extractions (words viewed as little-endian dwords: stream bit p is
            // bit p & 31 of dword p >> 5)
            const uint32_t *w32 = reinterpret_cast<const uint32_t *>(words);
            const int ht = matches32(bits32_at(w32, s), (uint32_t)W_HEAD, 12) +
                           matches32(bits32_at(w32, s + 500), (uint32_t)W_TAIL, 10);
            const uint32_t t22 = bits32_at(w32, s + 244);
            const int mn = ht + matches32(t22, (uint32_t)W_N, 22), mp = ht + matches32(t22, (uint32_t)W_P, 22);
            const int my = ht + matches32(bits32_at(w32, s + 214), (uint32_t)W_Y, 32) +
                           matches32(bits32_at(w32, s + 246), (uint32_t)(W_Y >> 32), 6);
            if (my >= 54) kind = 2;
            else if (mn >= 40 && mn >= mp) kind = 0;
            else if (mp >= 40) kind = 1;
        }
        const unsigned long long bal = __ballot(kind >= 0);
        if (bal) {
            const int first = __ffsll((long long)bal) - 1;
            const int k = __builtin_amdgcn_readlane(kind, first);   // first is wave-uniform
            if (lane == 0) { bstart[nb] = cur + first; bkind[nb] = k; }
            ++nb;
            cur = cur + first + 500;
            nextpos = cur;
        } else {
            cur += 64;
            nextpos = min(cur, nbits - 509);
        }
    }
    if (lead && ch < C) {   // the unconsumed tail
        int td0 = d0 + (nextpos >> 1), ph = nextpos & 1;
        int T = R + nd - td0;
        if (T > R) { td0 = nd; T = R; ph = 0; }   // (past ETSI_MAXB bursts only) keep the last R dibits
        if (T < 0) { td0 = R + nd; T = 0; ph = 0; }
        if (nhard) {   // other rows (double-buffered): moved here, the trellis reads only these rows
            tail_move(hard, soft, smax, ch, td0, T, ph, R, nhard, nsoft, lead, lane);
        } else if (lane == 0) {   // these rows: k_etsi_tail moves it after the trellis has read them
            tinfo[2 * ch] = td0;
            tinfo[2 * ch + 1] = (T << 1) | ph;
        }
    }
    __syncthreads();
    int per[3] = {0, 0, 0};
    if (lane == 0) {   // blocks per kind: normal-n 1 SCH/F; normal-p 2 SCH/HD; sync BSCH + SCH/HD
        for (int b = 0; b < nb; ++b) {
            if (bkind[b] == 0) ++per[0];
            else if (bkind[b] == 1) per[1] += 2;
            else { ++per[2]; ++per[1]; }
        }
        for (int k = 0; k < 3; ++k) per_all[wv][k] = per[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {   // the workgroup's three kind counters, packed 21 bits apart: one atomic
        unsigned long long inc = 0;
        for (int w = 0; w < SYNC_WAVES; ++w)
            inc += (unsigned long long)per_all[w][0] | ((unsigned long long)per_all[w][1] << 21) |
                   ((unsigned long long)per_all[w][2] << 42);
        block_old = inc ? atomicAdd(jcount, inc) : 0ull;
    }
    __syncthreads();
    if (lane == 0 && ch < C) {
        nburst[ch] = nb;
        nblock[ch] = per[0] + per[1] + per[2];
        int next[3];
        for (int k = 0; k < 3; ++k) {
            next[k] = (int)job_base(k, C) + (int)((block_old >> (21 * k)) & 0x1FFFFFull);
            for (int w = 0; w < wv; ++w) next[k] += per_all[w][k];
        }
        int q = 0;
        for (int b = 0; b < nb; ++b) {
            const int s = 2 * d0 + bstart[b], k = bkind[b];   // row bit (= the soft-bit row index)
            bursts[((size_t)ch * ETSI_MAXB + b) * 2] = s - 2 * R * (lead != nullptr);   // from the chunk's first new dibit
            bursts[((size_t)ch * ETSI_MAXB + b) * 2 + 1] = k;
            if (k == 0) {
                jobs[next[0]++] = Job{ch, q, b, 0, 0, s + 14}; ++q;
            } else if (k == 1) {
                jobs[next[1]++] = Job{ch, q, b, 0, 1, s + 14}; ++q;
                jobs[next[1]++] = Job{ch, q, b, 1, 1, s + 282}; ++q;
            } else {
                jobs[next[2]++] = Job{ch, q, b, 0, 2, s + 94}; ++q;
                jobs[next[1]++] = Job{ch, q, b, 1, 1, s + 282}; ++q;
            }
        }
    }
}


// Grid: one workgroup per SYNC_WAVES channels (the loop is a grid stride).
__global__ __launch_bounds__(64 * SYNC_WAVES) void k_etsi_sync(const uint8_t *__restrict__ hard, const int32_t *__restrict__ nsym,
                                                  int smax, int32_t *__restrict__ nburst, int32_t *__restrict__ bursts,
                                                  int32_t *__restrict__ nblock,
                                                  unsigned long long *__restrict__ jcount, Job *__restrict__ jobs,
                                                  int C, int32_t *lead, int R, int32_t *tinfo, const int8_t *soft,
                                                  uint8_t *nhard, int8_t *nsoft) {
    __shared__ SyncLds L;
    const int ng = (C + SYNC_WAVES - 1) / SYNC_WAVES;
    for (int g = blockIdx.x; g < ng; g += gridDim.x) {
        sync_group(L, g, hard, nsym, smax, nburst, bursts, nblock, jcount, jobs, C, lead, R, tinfo, soft, nhard,
                   nsoft);
        __syncthreads();   // L is reused by the next group
    }
}

__global__ __launch_bounds__(64) void k_etsi_tail(const uint8_t *__restrict__ hard, const int8_t *__restrict__ soft,
                                                  int stride, int C, const int32_t *__restrict__ tinfo, int R,
                                                  uint8_t *nhard, int8_t *nsoft, int32_t *__restrict__ lead) {
    const int ch = blockIdx.x;
    if (ch >= C) return;
    tail_move(hard, soft, stride, ch, tinfo[2 * ch], tinfo[2 * ch + 1] >> 1, tinfo[2 * ch + 1] & 1, R, nhard, nsoft,
              lead, threadIdx.x);
}

// --------------------------------------------------------------------------- E4 Viterbi
// Four LANES per coded block (one DPP quad) holding the 16 path metrics (layout below).  The quad loads
// the block's type-5 soft bits into one shared LDS row, descrambled (load_seg: 16 contiguous bytes
// per quad per load; the byte gather this replaced -- two scattered byte loads per soft bit -- was
// what the Viterbi cost the demod running beside it), and the trellis reads that row through the
// deinterleaver (acs_groups4); each lane packs its 4 decision bits of 8
// steps into one survivor dword ([group][job][lane], coalesced); all four lanes trace back (same
// path) and lane 0 writes the block with the CRC accumulated on the fly.  16 blocks per 64-lane
// workgroup keep LDS at 7 KB, so Viterbi workgroups fit beside the demod's on a CU.
constexpr int VROW = 436;   // LDS row per block: 432 type-3 values, padded to 109 dwords (bank spread)

template <int CTRL>
__device__ __forceinline__ int32_t quad_perm(int32_t v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}

// One contiguous segment of a block's type-5 soft bits (ND dwords) into the LDS row, descrambled.
// The quad reads the segment as aligned dwords, lane q taking dwords 4 i + q (16 contiguous bytes
// per quad per load), and realigns them with v_alignbyte, the next dword coming from the neighbour
// lane (quad rotate) or, for lane 3, from lane 0 of the next load.  A dword is loaded only if it
// starts at or before the buffer's last byte (`last`, a dword that holds it): a clamped load reads
// bytes the segment does not use.  Descrambling negates the int8 values whose scrambler byte is 1
// (four at a time: x ^ 0xFF + 1 per flagged byte, carry-free SWAR), as -v in int8 does.
// The loads go through buffer resources over the whole soft-bit buffer (sbr: from the dword that
// holds its first byte to the dword that holds its last) and the scrambler table (scr_r): one 32-bit
// offset per lane with the load index in the immediate field, where 64-bit clamped addresses held two
// VGPRs per load in flight; a load past the buffer returns 0 instead of the clamped dword (bytes the
// segment does not use either way).  seg_off: the segment's byte offset from sbr's base (whose
// alignment is the buffer's: sbr starts at a dword boundary), scr_off: the table segment's.
template <int ND>
__device__ __forceinline__ void load_seg(__amdgpu_buffer_rsrc_t sbr, uint32_t seg_off, __amdgpu_buffer_rsrc_t scr_r,
                                         uint32_t scr_off, uint32_t *d32, int q) {
    constexpr int NI = (ND + 1 + 3) / 4;   // loads per lane: dwords 0 .. ND of the aligned window
    const int sh = (int)(seg_off & 3);
    const uint32_t a0 = seg_off - sh + 4 * q, s0 = scr_off + 4 * q;
    uint32_t R[NI], S[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        R[i] = __builtin_amdgcn_raw_buffer_load_b32(sbr, a0 + 16 * i, 0, 0);
        S[i] = __builtin_amdgcn_raw_buffer_load_b32(scr_r, s0 + 16 * i, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int j = 4 * i + q;
        const uint32_t nq = (uint32_t)quad_perm<0x39>((int32_t)R[i]);   // lane (q + 1) & 3
        const uint32_t n0 = i + 1 < NI ? (uint32_t)quad_perm<0x00>((int32_t)R[i + 1]) : 0u;
        const uint32_t v = __builtin_amdgcn_alignbyte(q == 3 ? n0 : nq, R[i], (uint32_t)sh);
        const uint32_t m = S[i] * 0xFFu, x = v ^ m;   // scrambler bytes are 0 / 1
        const uint32_t dv = ((x & 0x7F7F7F7Fu) + (m & 0x01010101u)) ^ (x & 0x80808080u);
        if (j < ND) d32[j] = dv;
    }
}

// Strided state layout: lane l of the quad holds states n = 4 i + l in pm[i].  New state n has
// predecessors p0 = n >> 1 = 2 i + (l >> 1) (register i >> 1 of lane (2 i + (l >> 1)) & 3) and
// p1 = p0 | 8 (register (i >> 1) + 2, same lane): for a given i both sit in one register of a lane
// that one quad_perm pattern names, so each new metric takes two DPP moves and no selects.  The
// branch-metric signs depend on n & 3 = l (lane constants) and on n >> 2 = i (compile time).
// Survivors: a lane packs its 4 decision bits of 8 consecutive steps into one dword (bit
// 4 (t & 7) + i for state 4 i + l at step t) and stores it once per 8 steps, [group][job][lane]:
// one coalesced 256-B store per wave per 8 steps.
// The row holds the descrambled block in type-5 order; the deinterleaver is applied on the read:
// type-3 value i (1-based) is type-5 value k(i) = 1 + (A i mod K).  The index walk is the same for
// every lane of the wave (one block kind per wave), so it stays in scalar registers.
template <int GROUPS, int A, int K>
__device__ __forceinline__ void acs_groups4(int32_t (&pm)[4], int q, const int8_t *row, uint32_t *sv, size_t gstride) {
    // rate-2/3 puncturing: step 2g sees mother outputs (g1, g2) = type-3 (3g, 3g+1); step 2g+1 sees
    // g1 = type-3 3g+2; the other mother outputs are erased.
    const bool bb = q & 1, d0 = (q >> 1) & 1;   // bits 0 and 1 of this lane's states
    int r = 0;   // A i mod K for the type-3 value read last
    auto next = [&r]() {
        r += A;
        if (r >= K) r -= K;
        return r;
    };
    for (int gi = 0; gi < GROUPS; ++gi) {
        uint32_t word = 0;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int i0 = next(), i1 = next(), i2 = next();
            const int32_t a = row[i0], b = row[i1], c = row[i2];
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                // branch metric for d3 = 0 (d3 = 1 negates every generator output):
                // step 2g: +-a +-b (b's sign also flips with (n >> 2) ^ (n >> 3)); step 2g+1: +-c
                int32_t v0, v1;
                if (half == 0) {
                    const int32_t sa = (bb ^ d0) ? -a : a, sb = bb ? -b : b;
                    v0 = sa + sb;   // i with flip 0 (i = 0, 3)
                    v1 = sa - sb;   // flip 1 (i = 1, 2)
                } else {
                    v0 = v1 = (bb ^ d0) ? -c : c;
                }
                const int32_t X0 = quad_perm<0x50>(pm[0]), Y0 = quad_perm<0x50>(pm[2]);
                const int32_t X1 = quad_perm<0xFA>(pm[0]), Y1 = quad_perm<0xFA>(pm[2]);
                const int32_t X2 = quad_perm<0x50>(pm[1]), Y2 = quad_perm<0x50>(pm[3]);
                const int32_t X3 = quad_perm<0xFA>(pm[1]), Y3 = quad_perm<0xFA>(pm[3]);
                const int32_t X[4] = {X0, X1, X2, X3}, Y[4] = {Y0, Y1, Y2, Y3};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int32_t v = ((i ^ (i >> 1)) & 1) ? v1 : v0;
                    const int32_t m0 = X[i] + v, m1 = Y[i] - v;
                    const bool t1 = m1 > m0;
                    pm[i] = t1 ? m1 : m0;
                    word |= (uint32_t)t1 << (4 * (2 * g4 + half) + i);
                }
            }
        }
        sv[(size_t)gi * gstride] = word;
    }
}

// soft-bit and scrambler-table resources of one k_etsi_viterbi launch (wave-uniform)
struct VitSrc {
    __amdgpu_buffer_rsrc_t sbr, cell_r, bsch_r;
    uint32_t sb_lead;   // bytes from sbr's base (a dword boundary) to softbits[0]
};

template <int KIND>
__device__ __forceinline__ void viterbi_wave(int8_t *rows, const Job *__restrict__ jobs, int nj, size_t jbase, int lb,
                                             size_t ss, const VitSrc &src, int smax, uint32_t *__restrict__ surv) {
    constexpr KindP P = kind_params(KIND);
    const int lane = threadIdx.x, jw = lane >> 2, q = lane & 3;
    const int jl = lb * 16 + jw;
    if (lb * 16 >= nj) return;   // whole wave past this kind's job count
    const bool act = jl < nj;
    const size_t j = jbase + jl;
    const Job jb = act ? jobs[j] : Job{0, 0, 0, 0, KIND, 0};
    int8_t *row = rows + jw * VROW;
    if (act) {   // the quad loads the block's type-5 soft bits and scrambler bytes as dwords
        const uint32_t so = src.sb_lead + (uint32_t)jb.ch * 2 * smax + jb.off;
        const __amdgpu_buffer_rsrc_t scr_r = KIND == 2 ? src.bsch_r : src.cell_r;
        const uint32_t co = KIND == 2 ? 0u : (uint32_t)jb.ch * 432;
        uint32_t *d32 = (uint32_t *)row;
        if constexpr (KIND == 0) {   // SCH/F: BKN1 = type-5 [0, 216), BKN2 = [216, 432) 268 bits on
            load_seg<54>(src.sbr, so, scr_r, co, d32, q);
            load_seg<54>(src.sbr, so + 268, scr_r, co + 4 * 54, d32 + 54, q);
        } else {
            load_seg<P.K / 4>(src.sbr, so, scr_r, co, d32, q);
        }
    }
    __syncthreads();   // the quad's row (one wave per workgroup)
    int32_t pm[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) pm[m] = (q == 0 && m == 0) ? 0 : -(1 << 28);
    const size_t gstride = 4 * ss;   // dwords between survivor groups
    uint32_t *sv = surv + 4 * j + q;
    if (act) {
        constexpr int NG = P.n2 / 8;   // n2 is a multiple of 8
        acs_groups4<NG, P.a, P.K>(pm, q, row, sv, gstride);
    }
}

// Traceback + CRC of one block per LANE (k_etsi_traceback): 64 blocks per wave, a quarter of the
// wave instructions the quad-per-block trellis waves would spend on the same serial chain (all four
// lanes of a quad followed the same path).  From state 0 (tail bits); a group's four survivor words
// ([group][job][lane]) are one 16-B load, eight groups (64 steps) in flight; the CRC over type-1 +
// CRC bits accumulates on the fly; type-1 bits go out four per dword store.
template <int KIND>
__device__ __forceinline__ void traceback_lane(const Job &jb, const uint32_t *__restrict__ sv, size_t gstride,
                                               int32_t *__restrict__ blocks, uint8_t *__restrict__ type1) {
    constexpr KindP P = kind_params(KIND);
    constexpr int NG = P.n2 / 8;
    constexpr int L = P.n1 + 16;
    static_assert(P.n1 % 4 == 0, "type-1 bits stored four per dword");
    uint32_t c = CRC_TAB.init[L];
    int s2 = 0;
    uint32_t acc = 0;
    uint8_t *ob = type1 + ((size_t)jb.ch * ETSI_MAXJ + jb.slot) * 268;
    uint32_t *op = (uint32_t *)ob;
    const bool al4 = ((uintptr_t)type1 & 3) == 0;   // a caller's device pointer may be unaligned
    for (int g0 = NG - 1; g0 >= 0; g0 -= 8) {
        uint4 w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = *(const uint4 *)(sv + (size_t)max(g0 - u, 0) * gstride);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int gi = g0 - u;
            if (gi < 0) break;
#pragma unroll
            for (int st = 7; st >= 0; --st) {
                const int t = 8 * gi + st;
                const uint32_t bit = s2 & 1;
                acc = (acc << 8) | bit;
                if ((st & 3) == 0 && t < P.n1) {   // bytes t .. t+3
                    if (al4) {
                        op[t >> 2] = acc;
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; ++k) ob[t + k] = (uint8_t)(acc >> (8 * k));
                    }
                }
                // unconditional, wave-uniform table read (scalar load, hoisted); a per-lane branch
                // around it made every step wait a global load
                const uint32_t tv = CRC_TAB.t[L - 1 - t < 0 ? 0 : L - 1 - t];
                c ^= tv & (0u - (bit & (uint32_t)(t < L)));
                // state s2's decision: word of lane s2 & 3, bit 4 st + (s2 >> 2)
                const int ln = s2 & 3;
                const uint32_t ww = ln & 2 ? (ln & 1 ? w[u].w : w[u].z) : (ln & 1 ? w[u].y : w[u].x);
                s2 = (s2 >> 1) | ((int)((ww >> (4 * st + (s2 >> 2))) & 1u) << 3);
            }
        }
    }
    int32_t *bm = blocks + ((size_t)jb.ch * ETSI_MAXJ + jb.slot) * 4;
    bm[0] = KIND;   // four dword stores: the caller's pointer need not be 16-B aligned
    bm[1] = c == 0x1D0Fu;
    bm[2] = jb.burst;
    bm[3] = jb.blk;
}

// Grid: the SCH/F region's waves, then SCH/HD's, then BSCH's (one trellis length per wave).
__global__ __launch_bounds__(64) void k_etsi_viterbi(const Job *__restrict__ jobs,
                                                     const unsigned long long *__restrict__ jcount, int C,
                                                     const int8_t *__restrict__ softbits, int smax,
                                                     const uint8_t *__restrict__ cell_scr,
                                                     const uint8_t *__restrict__ bsch_scr,
                                                     uint32_t *__restrict__ surv, int kmask) {
    __shared__ __attribute__((aligned(16))) int8_t rows[16 * VROW];
    const size_t ss = 32 * (size_t)C;
    // the soft-bit buffer [softbits, softbits + 2 C smax) from the dword holding its first byte to the
    // dword holding its last (host checks: < 4 GiB); the cell table and the BSCH table
    const uintptr_t sb0 = (uintptr_t)softbits & ~(uintptr_t)3;
    const uintptr_t sbl = ((uintptr_t)softbits + (size_t)C * 2 * smax - 1) & ~(uintptr_t)3;
    VitSrc src;
    src.sbr = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(sb0), 0, (int)(sbl - sb0 + 4), 0x00020000);
    src.cell_r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(cell_scr), 0, C * 432, 0x00020000);
    src.bsch_r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(bsch_scr), 0, 432, 0x00020000);
    src.sb_lead = (uint32_t)((uintptr_t)softbits - sb0);
    const unsigned long long cnt = *jcount;
    // kinds outside kmask are left to another launch (cell acquisition decodes BSCH first)
    const int n0 = kmask & 1 ? (int)(cnt & 0x1FFFFFull) : 0, n1 = kmask & 2 ? (int)((cnt >> 21) & 0x1FFFFFull) : 0,
              n2 = kmask & 4 ? (int)(cnt >> 42) : 0;
    // the waves the job counts need (16 blocks each), walked with a grid stride: a grid smaller
    // than that keeps the lower MAC's LDS beside the demod's bounded when the two run side by side
    const int nb0 = (n0 + 15) / 16, nb1 = (n1 + 15) / 16, nb2 = (n2 + 15) / 16;
    for (int b = blockIdx.x; b < nb0 + nb1 + nb2; b += gridDim.x) {
        if (b < nb0)
            viterbi_wave<0>(rows, jobs, n0, job_base(0, C), b, ss, src, smax, surv);
        else if (b < nb0 + nb1)
            viterbi_wave<1>(rows, jobs, n1, job_base(1, C), b - nb0, ss, src, smax, surv);
        else
            viterbi_wave<2>(rows, jobs, n2, job_base(2, C), b - nb0 - nb1, ss, src, smax, surv);
        __syncthreads();   // rows are rewritten by the next wave-batch
    }
}

// One lane per block (64 per wave), the kinds' regions one after another; grid stride as above.
__global__ __launch_bounds__(64) void k_etsi_traceback(const Job *__restrict__ jobs,
                                                       const unsigned long long *__restrict__ jcount, int C,
                                                       const uint32_t *__restrict__ surv,
                                                       int32_t *__restrict__ blocks, uint8_t *__restrict__ type1,
                                                       int kmask) {
    const size_t gstride = 4 * 32 * (size_t)C;   // dwords between survivor groups
    const unsigned long long cnt = *jcount;
    const int n[3] = {kmask & 1 ? (int)(cnt & 0x1FFFFFull) : 0, kmask & 2 ? (int)((cnt >> 21) & 0x1FFFFFull) : 0,
                      kmask & 4 ? (int)(cnt >> 42) : 0};
    const int nb0 = (n[0] + 63) / 64, nb1 = (n[1] + 63) / 64, nb2 = (n[2] + 63) / 64;
    for (int b = blockIdx.x; b < nb0 + nb1 + nb2; b += gridDim.x) {
        const int kind = b < nb0 ? 0 : b < nb0 + nb1 ? 1 : 2;
        const int jl = 64 * (b - (kind == 0 ? 0 : kind == 1 ? nb0 : nb0 + nb1)) + (int)threadIdx.x;
        if (jl >= n[kind]) continue;
        const size_t j = job_base(kind, C) + jl;
        const Job jb = jobs[j];
        const uint32_t *sv = surv + 4 * j;
        if (kind == 0) traceback_lane<0>(jb, sv, gstride, blocks, type1);
        else if (kind == 1) traceback_lane<1>(jb, sv, gstride, blocks, type1);
        else traceback_lane<2>(jb, sv, gstride, blocks, type1);
    }
}

// --------------------------------------------------------------------------- cell acquisition
// One lane per channel, after the BSCH blocks of the chunk are decoded (colour code 0): the last
// CRC-good BSCH of the channel gives its extended colour code -- MAC-SYNC colour code at type-1
// bits 4..9, D-MLE-SYNC MCC at 31..40 and MNC at 41..54 (EN 300 392-2 §21.4.4.2, §18.4.2.1) -- and
// the scrambling init (ecc << 2) | 3 (§8.2.5.2).  Without one the channel keeps its init.  The
// channel's 432 scrambler bytes (the table k_etsi_viterbi descrambles with) are regenerated only
// when the init differs from the one the table was made for (tab_init; 0 = none yet).
constexpr uint32_t SCR_TAPS = (1u << 0) | (1u << 6) | (1u << 9) | (1u << 10) | (1u << 16) | (1u << 20) | (1u << 21) |
                              (1u << 22) | (1u << 24) | (1u << 25) | (1u << 27) | (1u << 28) | (1u << 30) | (1u << 31);

__global__ __launch_bounds__(256) void k_cell_acquire(int C, const int32_t *__restrict__ nburst,
                                                      const int32_t *__restrict__ bursts,
                                                      const int32_t *__restrict__ blocks,
                                                      const uint8_t *__restrict__ type1, uint32_t *__restrict__ cell_init,
                                                      uint32_t *__restrict__ tab_init, uint8_t *__restrict__ cell_scr) {
    const int ch = blockIdx.x * 256 + threadIdx.x;
    if (ch >= C) return;
    uint32_t init = cell_init[ch];
    const int nb = min(nburst[ch], ETSI_MAXB);
    int q = 0;   // block slot of burst b: the sync kernel's numbering (1 per NDB(n), 2 per NDB(p) / SB)
    for (int b = 0; b < nb; ++b) {
        const int k = bursts[((size_t)ch * ETSI_MAXB + b) * 2 + 1];
        if (k == 2 && q < ETSI_MAXJ && blocks[((size_t)ch * ETSI_MAXJ + q) * 4 + 1]) {
            const uint8_t *t = type1 + ((size_t)ch * ETSI_MAXJ + q) * 268;
            uint32_t ecc = 0;
            for (int i = 4; i < 10; ++i) ecc = (ecc << 1) | (t[i] & 1u);     // colour code (low 6)
            uint32_t mm = 0;
            for (int i = 31; i < 55; ++i) mm = (mm << 1) | (t[i] & 1u);     // MCC(10) MNC(14)
            init = (((mm << 6) | ecc) << 2) | 3u;
        }
        q += k == 0 ? 1 : 2;
    }
    cell_init[ch] = init;
    if (tab_init[ch] != init) {
        tab_init[ch] = init;
        uint32_t r = init;
        uint32_t *o = reinterpret_cast<uint32_t *>(cell_scr + (size_t)ch * 432);
        for (int w = 0; w < 108; ++w) {   // four scrambler bytes (0 / 1) per dword store
            uint32_t v = 0;
            for (int k = 0; k < 4; ++k) {
                const uint32_t bt = (uint32_t)__popc(r & SCR_TAPS) & 1u;
                r = (r >> 1) | (bt << 31);
                v |= bt << (8 * k);
            }
            o[w] = v;
        }
    }
}

// ETSI differential decision on given symbol-spaced samples (SignalProcessor(mode="etsi")
// .demodulate_dqpsk): d = x[k] conj(x[k-1]), dibit = (Im d < 0, Re d < 0) -- EN 300 392-2 Table 5.1
// (00 +pi/4, 01 +3pi/4, 11 -3pi/4, 10 -pi/4), the fused demod's decision without its CFO rotation.
template <typename T>
__global__ __launch_bounds__(256) void k_etsi_decide(const T *__restrict__ x, long n, uint8_t *__restrict__ hard) {
    const long k = (long)blockIdx.x * 256 + threadIdx.x + 1;
    if (k >= n) return;
    const float ar = (float)x[k].x, ai = (float)x[k].y, br = (float)x[k - 1].x, bi = (float)x[k - 1].y;
    const float dr = fmaf(ar, br, ai * bi), di = fmaf(ai, br, -(ar * bi));
    hard[k - 1] = (uint8_t)(((di < 0.0f) << 1) | (dr < 0.0f));
}

// --------------------------------------------------------------------------- component kernels
// Block decode of F independent blocks of one kind (16 lanes per block, 4 per wave).
__global__ __launch_bounds__(64) void k_decode_blocks(const int8_t *__restrict__ soft5, int F, int kind,
                                                      const uint8_t *__restrict__ scr /*[F][K]*/,
                                                      uint8_t *__restrict__ type1, uint8_t *__restrict__ crc_ok) {
    __shared__ __attribute__((aligned(16))) int8_t ms[4][4 * 288];
    __shared__ uint64_t surv[288];
    __shared__ uint8_t t2[4][288];
    const int lane = threadIdx.x, g = lane >> 4, st = lane & 15;
    const int j = blockIdx.x * 4 + g;
    const bool act = j < F;
    const KindP P = kind_params(kind);
    for (int i = st; i < 4 * P.n2; i += 16) ms[g][i] = 0;
    __syncthreads();
    if (act) {
        for (int i = 1 + st; i <= P.K; i += 16) {
            const int k = 1 + (int)(((long)P.a * i) % P.K);
            const int8_t v = soft5[(size_t)j * P.K + k - 1];
            ms[g][punct_index(i) - 1] = scr[(size_t)j * P.K + k - 1] ? (int8_t)(-v) : v;
        }
    }
    __syncthreads();
    int32_t pm = st == 0 ? 0 : -(1 << 28);
    const int b = st & 1, d0 = (st >> 1) & 1, d1 = (st >> 2) & 1, d2 = (st >> 3) & 1;
    for (int t = 0; t < P.n2; ++t) {
        const int8_t *m = ms[g] + 4 * t;
        const int32_t m0 = m[0], m1 = m[1], m2 = m[2], m3 = m[3];
        const int32_t v0 = ((b ^ d0) ? -m0 : m0) + ((b ^ d1 ^ d2) ? -m1 : m1) + ((b ^ d0 ^ d1) ? -m2 : m2) +
                           ((b ^ d0 ^ d2) ? -m3 : m3);
        const int32_t a0 = __shfl(pm, (lane & ~15) + (st >> 1), 64) + v0;
        const int32_t a1 = __shfl(pm, (lane & ~15) + ((st >> 1) | 8), 64) - v0;
        const bool take1 = a1 > a0;
        const unsigned long long sv = __ballot(take1);
        pm = take1 ? a1 : a0;
        if (lane == 0) surv[t] = sv;
    }
    __syncthreads();
    if (act && st == 0) {
        int s2 = 0;
        for (int t = P.n2 - 1; t >= 0; --t) {
            t2[g][t] = (uint8_t)(s2 & 1);
            s2 = (s2 >> 1) | ((int)((surv[t] >> (16 * g + s2)) & 1ull) << 3);
        }
        uint32_t c = 0xFFFF;
        for (int i = 0; i < P.n1 + 16; ++i) {
            c ^= (uint32_t)t2[g][i] << 15;
            c = (c & 0x8000u) ? ((c << 1) ^ 0x1021u) : (c << 1);
            c &= 0xFFFFu;
        }
        crc_ok[j] = c == 0x1D0Fu;
    }
    __syncthreads();
    if (act)
        for (int i = st; i < P.n1; i += 16) type1[(size_t)j * P.n1 + i] = t2[g][i];
}

// Encoder type-1 -> type-5 (one block per thread; CRC, tail, mother code, puncture, interleave, scramble)
__global__ void k_encode_blocks(const uint8_t *__restrict__ type1, int F, int kind, const uint8_t *__restrict__ scr,
                                uint8_t *__restrict__ type5) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= F) return;
    const KindP P = kind_params(kind);
    const uint8_t *in = type1 + (size_t)j * P.n1;
    uint8_t t2[288];
    uint32_t c = 0xFFFF;
    for (int i = 0; i < P.n1; ++i) {
        t2[i] = in[i] & 1;
        c ^= (uint32_t)t2[i] << 15;
        c = (c & 0x8000u) ? ((c << 1) ^ 0x1021u) : (c << 1);
        c &= 0xFFFFu;
    }
    c ^= 0xFFFFu;
    for (int k = 0; k < 16; ++k) t2[P.n1 + k] = (c >> (15 - k)) & 1u;
    for (int k = 0; k < 4; ++k) t2[P.n1 + 16 + k] = 0;
    for (int i = 1; i <= P.K; ++i) {
        const int mi = punct_index(i) - 1;   // mother index: step mi/4, generator mi%4
        const int step = mi >> 2, gen = mi & 3;
        const uint32_t bb = t2[step];
        const uint32_t e0 = step >= 1 ? t2[step - 1] : 0, e1 = step >= 2 ? t2[step - 2] : 0,
                       e2 = step >= 3 ? t2[step - 3] : 0, e3 = step >= 4 ? t2[step - 4] : 0;
        uint32_t v = gen == 0 ? (bb ^ e0 ^ e3) : gen == 1 ? (bb ^ e1 ^ e2 ^ e3) : gen == 2 ? (bb ^ e0 ^ e1 ^ e3)
                                                                                          : (bb ^ e0 ^ e2 ^ e3);
        const int k = 1 + (int)(((long)P.a * i) % P.K);
        type5[(size_t)j * P.K + k - 1] = (uint8_t)(v ^ scr[(size_t)j * P.K + k - 1]);
    }
}

}  // namespace

// A streaming window too short for the channel filter (M2 <= 0): no symbols, the acquired loops'
// positions move to the end of the (empty) window (track_store's M2 < 16 rule).
__global__ __launch_bounds__(256) void k_track_skip(tetra_etsi_track *__restrict__ tr, int C, int yoff, int M2) {
    const int ch = blockIdx.x * 256 + threadIdx.x;
    if (ch < C && tr[ch].acquired) tr[ch].base = tr[ch].base + (float)(yoff - M2);
}

// --------------------------------------------------------------------------- host side
static void scramble_seq(uint32_t r, int n, uint8_t *out) {
    for (int i = 0; i < n; ++i) {
        const uint32_t b = ((r >> 0) ^ (r >> 6) ^ (r >> 9) ^ (r >> 10) ^ (r >> 16) ^ (r >> 20) ^ (r >> 21) ^ (r >> 22) ^
                            (r >> 24) ^ (r >> 25) ^ (r >> 27) ^ (r >> 28) ^ (r >> 30) ^ (r >> 31)) & 1u;
        r = (r >> 1) | (b << 31);
        out[i] = (uint8_t)b;
    }
}

// The canonical 2.4 MSps plan runs on the fused per-wave kernels; any other supported plan (or a
// canonical one with TETRA_ETSI_FORCE_GENERIC) on the generic-rate channel filter (etsi_rate.hip).
static bool canonical(const tetra_etsi_plan *P) {
    return P->q1 == 10 && P->L1 == 48 && P->up == 3 && P->down == 10 && P->Lp == 3 * TPP &&
           !(P->flags & TETRA_ETSI_FORCE_GENERIC);
}
static int etsi_check(tetra_ctx *ctx, const tetra_etsi_plan *P) {
    if (!P) return tetra_fail(ctx, TETRA_E_INVALID, "plan is NULL");
    if (canonical(P)) return TETRA_OK;
    if (const char *why = etsi_generic_unsupported(P))
        return tetra_fail(ctx, TETRA_E_INVALID, "unsupported ETSI plan: %s", why);
    return TETRA_OK;
}

// Which channel-filter kernel a launch takes (launch_chanfilt, tetra_etsi_kernel_info).
enum CfKernel { CF_R_FUSED, CF_R, CF_SC16_FUSED, CF_SC16, CF_F4_FUSED, CF_F4 };
// the per-wave filter (k_chanfilt_r): y in LDS (M2 <= YLDS); SC16 rows of whole 16-B loads
static bool per_wave(int fmt, int64_t M2, size_t N) { return M2 <= YLDS && (fmt == TETRA_CF32 || N % 4 == 0); }
// the fused demod's condition: y (and the tail's staging) fit the kernel's LDS
static bool fused_fits(int fmt, int64_t M2, int64_t sm, size_t N) {
    if (!per_wave(fmt, M2, N)) return fmt == TETRA_SC16 && M2 + sm <= CF_LDS2_SC16;
    return sm <= WTAIL_SM;
}
static CfKernel chanfilt_kernel(int fmt, int64_t M2, size_t N, bool fused) {
    if (per_wave(fmt, M2, N)) return fused ? CF_R_FUSED : CF_R;
    if (fmt == TETRA_SC16) return fused ? CF_SC16_FUSED : CF_SC16;
    return fused ? CF_F4_FUSED : CF_F4;
}
static const void *chanfilt_fn(CfKernel k, int fmt) {
    const bool cf = fmt == TETRA_CF32;
    switch (k) {
    case CF_R_FUSED:
        return cf ? reinterpret_cast<const void *>(&k_chanfilt_r<float4, true>)
                  : reinterpret_cast<const void *>(&k_chanfilt_r<uint4, true>);
    case CF_R:
        return cf ? reinterpret_cast<const void *>(&k_chanfilt_r<float4, false>)
                  : reinterpret_cast<const void *>(&k_chanfilt_r<uint4, false>);
    case CF_SC16_FUSED: return reinterpret_cast<const void *>(&k_chanfilt<uint2, true>);
    case CF_SC16: return reinterpret_cast<const void *>(&k_chanfilt<uint2, false>);
    case CF_F4_FUSED: return reinterpret_cast<const void *>(&k_chanfilt<float4, true>);
    default: return reinterpret_cast<const void *>(&k_chanfilt<float4, false>);
    }
}
static const char *const CF_NAMES[] = {"k_chanfilt_r", "k_chanfilt_r", "k_chanfilt", "k_chanfilt", "k_chanfilt",
                                       "k_chanfilt"};

// Stage-1 taps and the per-branch stage-2 tap table (k_chanfilt), then the launch.
static int launch_chanfilt(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *x, int fmt, size_t C, size_t N,
                           int64_t M1, int64_t M2, float2 *y, const TimingOut *fused = nullptr, size_t ld = 0,
                           size_t Nk = 0) {
    if (ld == 0) ld = N;   // row pitch in samples (streaming windows inside a resident capture: > N)
    if (Nk == 0) Nk = N;   // the length the kernel choice sees (N + 1 keeps SC16 off the per-wave kernel)
    if (!canonical(P)) return fused ? TETRA_E_INVALID : launch_chanfilt_generic(ctx, P, x, fmt, C, N, M1, M2, y, ld);
    static_assert(sizeof(ctx->coef_etsi) == CF_COEF * sizeof(float), "tap image size");
    float *coef = (float *)ws(ctx, S_W12, CF_COEF * 4);   // slot of its own: the image persists
    if (!coef) return TETRA_E_NOMEM;
    float hc[CF_COEF];
    static const int i0[3] = {320, 318, 319}, off[3] = {0, 4, 7};
    for (int j = 0; j < 64; ++j) {
        hc[j] = j < 48 ? P->h1[j] : 0.f;
        hc[64 + j] = hc[j] * (1.0f / 32768.0f);   // k_chanfilt_r's SC16 taps: the sample scale folded in (exact)
    }
    // A fragment of k-step ks for lane l: A[i = l & 15][s = 4 ks + (l >> 4)], row i = 3q + c
    for (int ks = 0; ks < S2K; ++ks)
        for (int l = 0; l < 64; ++l) {
            const int i = l & 15, sidx = 4 * ks + (l >> 4), q = i / 3, c = i % 3;
            const int j = sidx - 10 * q - off[c];
            hc[128 + 64 * ks + l] = i < 15 && j >= 0 && j < TPP ? P->hp[i0[c] - 3 * j] : 0.f;
        }
    // upload only when the taps or the workspace changed: a per-call pageable copy would sit on the
    // stream in front of every launch
    if (ctx->coef_etsi_dev != coef || memcmp(hc, ctx->coef_etsi, sizeof(hc)) != 0) {
        memcpy(ctx->coef_etsi, hc, sizeof(hc));
        HIP_TRY(ctx, hipMemcpyAsync(coef, ctx->coef_etsi, CF_COEF * 4, hipMemcpyHostToDevice, ctx->stream));
        ctx->coef_etsi_dev = coef;
    }
    const CfKernel kind = chanfilt_kernel(fmt, M2, Nk, fused != nullptr);
    PROF(ctx, fused ? "etsi_demod" : "etsi_chanfilt");
    const TimingOut to = fused ? *fused : TimingOut{};
    const dim3 g((unsigned)C), b(256);
    switch (kind) {
    case CF_R_FUSED:
        if (fmt == TETRA_CF32)
            hipLaunchKernelGGL((k_chanfilt_r<float4, true>), g, b, 0, ctx->stream, (const float4 *)x, (long)N, (int)M1,
                               (int)M2, coef, coef + 128, y, to, (long)ld);
        else
            hipLaunchKernelGGL((k_chanfilt_r<uint4, true>), g, b, 0, ctx->stream, (const uint4 *)x, (long)N, (int)M1,
                               (int)M2, coef + 64, coef + 128, y, to, (long)ld);
        break;
    case CF_R:
        if (fmt == TETRA_CF32)
            hipLaunchKernelGGL((k_chanfilt_r<float4, false>), g, b, 0, ctx->stream, (const float4 *)x, (long)N, (int)M1,
                               (int)M2, coef, coef + 128, y, to, (long)ld);
        else
            hipLaunchKernelGGL((k_chanfilt_r<uint4, false>), g, b, 0, ctx->stream, (const uint4 *)x, (long)N, (int)M1,
                               (int)M2, coef + 64, coef + 128, y, to, (long)ld);
        break;
    case CF_SC16_FUSED:
        hipLaunchKernelGGL((k_chanfilt<uint2, true>), g, b, 0, ctx->stream, (const uint2 *)x, (long)N, (int)M1, (int)M2,
                           coef, coef + 128, y, to, (long)ld);
        break;
    case CF_SC16:
        hipLaunchKernelGGL((k_chanfilt<uint2, false>), g, b, 0, ctx->stream, (const uint2 *)x, (long)N, (int)M1,
                           (int)M2, coef, coef + 128, y, to, (long)ld);
        break;
    case CF_F4_FUSED:
        hipLaunchKernelGGL((k_chanfilt<float4, true>), g, b, 0, ctx->stream, (const float4 *)x, (long)N, (int)M1,
                           (int)M2, coef, coef + 128, y, to, (long)ld);
        break;
    default:
        hipLaunchKernelGGL((k_chanfilt<float4, false>), g, b, 0, ctx->stream, (const float4 *)x, (long)N, (int)M1,
                           (int)M2, coef, coef + 128, y, to, (long)ld);
    }
    HIP_TRY(ctx, hipGetLastError());
    return TETRA_OK;
}

extern "C" {

int tetra_etsi_lengths(const tetra_etsi_plan *P, size_t N, int64_t *M1, int64_t *M2, int64_t *smax) {
    if (!P || !M1 || !M2 || !smax) return TETRA_E_INVALID;
    long m1 = N >= (size_t)P->L1 ? ((long)N - P->L1) / P->q1 + 1 : 0;
    long m2 = (P->up * m1 - 1 - (P->Lp - 1)) >= 0 ? (P->up * m1 - 1 - (P->Lp - 1)) / P->down + 1 : 0;
    *M1 = m1;
    *M2 = m2;
    *smax = m2 / 4 + 2;
    return TETRA_OK;
}

int tetra_etsi_kernel_info(tetra_ctx *ctx, const tetra_etsi_plan *P, int fmt, size_t N, int fused, char *name,
                           size_t name_len, int64_t *lds_bytes) {
    if (!ctx || !P || (fmt != TETRA_CF32 && fmt != TETRA_SC16)) return TETRA_E_INVALID;
    int64_t M1, M2, sm;
    tetra_etsi_lengths(P, N, &M1, &M2, &sm);
    hipFuncAttributes a;
    if (etsi_check(ctx, P)) return TETRA_E_INVALID;
    if (!canonical(P)) {
        HIP_TRY(ctx, hipFuncGetAttributes(&a, chanfilt_generic_fn(fmt)));
        if (name && name_len) snprintf(name, name_len, "%s", "k_chanfilt_g");
        if (lds_bytes) *lds_bytes = (int64_t)a.sharedSizeBytes;
        return TETRA_OK;
    }
    if (fused) fused = fused_fits(fmt, M2, sm, N);   // the fused form's own condition (tetra_demod_etsi_fmt)
    const CfKernel k = chanfilt_kernel(fmt, M2, N, fused != 0);
    HIP_TRY(ctx, hipFuncGetAttributes(&a, chanfilt_fn(k, fmt)));
    if (name && name_len) snprintf(name, name_len, "%s", CF_NAMES[k]);
    if (lds_bytes) *lds_bytes = (int64_t)a.sharedSizeBytes;
    return TETRA_OK;
}

int tetra_etsi_set_cells(tetra_ctx *ctx, const uint32_t *scramb_init, size_t C) {
    if (!ctx || !scramb_init || C == 0) return TETRA_E_INVALID;
    std::vector<uint32_t> init(C);
    HIP_TRY(ctx, hipMemcpy(init.data(), scramb_init, C * 4, hipMemcpyDefault));
    std::vector<uint8_t> tab(C * 432 + 432);
    for (size_t c = 0; c < C; ++c) scramble_seq(init[c], 432, tab.data() + c * 432);
    scramble_seq(3u, 432, tab.data() + C * 432);   // BSCH: colour code 0
    uint8_t *d = (uint8_t *)ws(ctx, S_W5, tab.size());
    uint32_t *ti = (uint32_t *)ws(ctx, S_W14, C * 4);   // the inits the table holds (cell acquisition)
    if (!d || !ti) return TETRA_E_NOMEM;
    HIP_TRY(ctx, hipMemcpyAsync(d, tab.data(), tab.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ti, init.data(), C * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->cells = C;
    return TETRA_OK;
}

int tetra_etsi_chanfilt(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *iq, size_t C, size_t N, void *y) {
    return tetra_etsi_chanfilt_fmt(ctx, P, iq, TETRA_CF32, C, N, y);
}

int tetra_etsi_chanfilt_fmt(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *iq, int fmt, size_t C, size_t N,
                            void *y) {
    if (!ctx) return TETRA_E_INVALID;
    int rc = etsi_check(ctx, P);
    if (rc) return rc;
    if (N % 2 || C == 0) return tetra_fail(ctx, TETRA_E_INVALID, "N must be even");
    if (fmt != TETRA_CF32 && fmt != TETRA_SC16) return tetra_fail(ctx, TETRA_E_INVALID, "iq_fmt must be cf32 or sc16");
    int64_t M1, M2, smax;
    tetra_etsi_lengths(P, N, &M1, &M2, &smax);
    if (M2 <= 0) return tetra_fail(ctx, TETRA_E_INVALID, "chunk too short for the channel filter");
    Staging st(ctx);
    const void *x = st.in(iq, C * N * (fmt == TETRA_SC16 ? 4 : 8));
    void *yo = st.out(y, C * (size_t)M2 * 8);
    if (!x || !yo) return st.finish();
    rc = launch_chanfilt(ctx, P, x, fmt, C, N, M1, M2, (float2 *)yo);
    if (rc) return rc;
    return st.finish();
}

int tetra_etsi_timing(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *y, size_t C, size_t M2, void *soft,
                      int8_t *softbits, uint8_t *hard, int32_t *nsym, size_t smax, float *diag) {
    if (!ctx || !P || C == 0) return TETRA_E_INVALID;
    Staging st(ctx);
    const void *yd = st.in(y, C * M2 * 8);
    void *so = st.out(soft, C * smax * 8);
    int8_t *sbo = (int8_t *)st.out(softbits, C * smax * 2);
    uint8_t *ho = (uint8_t *)st.out(hard, C * smax);
    int32_t *no = (int32_t *)st.out(nsym, C * 4);
    float *dg = diag ? (float *)st.out(diag, C * 16) : nullptr;
    float2 *dscr = (float2 *)ws(ctx, S_W4, C * smax * 8);
    if (!yd || !so || !sbo || !ho || !no || !dscr) return st.finish();
    {
        PROF(ctx, "etsi_timing");
        hipLaunchKernelGGL(timing_kernel(M2, smax), dim3((unsigned)C), dim3(64), 0, ctx->stream, (const float2 *)yd, (int)M2, P->gain,
                           P->soft_scale, (float2 *)so, dscr, sbo, ho, no, (int)smax, (float4 *)dg, timing_probe(),
                           nullptr, 0, 0, 0, nullptr, 0, 0, 0, 0);
    }
    return st.finish();
}

// The chunked timing both wideband entry points launch (cstride = the chunk stride, rowlen = the
// carrier rows' length): tetra_etsi_timing_om's chunks tile the rows, tetra_etsi_timing_chunks' overlap.
static int launch_timing_chunks(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *y, size_t M, size_t rowlen,
                                size_t nchunk, size_t stride, size_t len, const void *om, size_t ngrp, int U,
                                void *soft, int8_t *softbits, uint8_t *hard, int32_t *nsym, size_t smax, float *diag) {
    const size_t C = M * nchunk;
    Staging st(ctx);
    const void *yd = st.in(y, M * rowlen * 8);
    const void *omd = om ? st.in(om, M * ngrp * 16) : nullptr;
    void *so = st.out(soft, C * smax * 8);
    int8_t *sbo = (int8_t *)st.out(softbits, C * smax * 2);
    uint8_t *ho = (uint8_t *)st.out(hard, C * smax);
    int32_t *no = (int32_t *)st.out(nsym, C * 4);
    float *dg = diag ? (float *)st.out(diag, C * 16) : nullptr;
    // the grouped form needs no d_j scratch: the LEAN form recomputes d_j from the stored symbols
    float2 *dscr = om ? nullptr : (float2 *)ws(ctx, S_W4, C * smax * 8);
    if (!yd || (om && !omd) || !so || !sbo || !ho || !no || (!om && !dscr)) return st.finish();
    {
        PROF(ctx, "etsi_timing");
        hipLaunchKernelGGL(timing_kernel(len, smax, om != nullptr), dim3((unsigned)C), dim3(64), 0, ctx->stream,
                           (const float2 *)yd, (int)len, P->gain, P->soft_scale, (float2 *)so, dscr, sbo, ho, no,
                           (int)smax, (float4 *)dg, timing_probe(), (const float4 *)omd, (int)nchunk, (int)ngrp, U,
                           nullptr, 0, 0, (int)stride, (long)rowlen);
    }
    return st.finish();
}

int tetra_etsi_timing_om(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *y, size_t C, size_t M2,
                         const void *om, size_t nchunk, size_t ngrp, int U, void *soft, int8_t *softbits,
                         uint8_t *hard, int32_t *nsym, size_t smax, float *diag) {
    if (!ctx || !P || C == 0 || !om) return TETRA_E_INVALID;
    if (nchunk == 0 || C % nchunk || M2 % 4 || U < 4 || U > 64 || U % 4 || ngrp * (size_t)U < nchunk * M2 ||
        M2 < 16 || nchunk * M2 * 8 >= ((size_t)1 << 31))
        return tetra_fail(ctx, TETRA_E_INVALID, "timing_om: C a multiple of nchunk, M2 >= 16 a multiple of 4, "
                                                "4 <= U <= 64 a multiple of 4, ngrp U >= nchunk M2");
    return launch_timing_chunks(ctx, P, y, C / nchunk, nchunk * M2, nchunk, M2, M2, om, ngrp, U, soft, softbits, hard,
                                nsym, smax, diag);
}

int tetra_etsi_timing_chunks(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *y, size_t M, size_t rowlen,
                             size_t nchunk, size_t stride, size_t len, const void *om, size_t ngrp, int U, void *soft,
                             int8_t *softbits, uint8_t *hard, int32_t *nsym, size_t smax, float *diag) {
    if (!ctx || !P || M == 0) return TETRA_E_INVALID;
    if (nchunk == 0 || stride == 0 || len < 16 || (nchunk - 1) * stride + 16 > rowlen ||
        rowlen * 8 >= ((size_t)1 << 31) || M * nchunk > INT32_MAX || smax < len / 4 + 2)
        return tetra_fail(ctx, TETRA_E_INVALID, "timing_chunks: nchunk >= 1, stride >= 1, len >= 16, every chunk "
                                                ">= 16 samples of the row, rows < 2^28 samples, smax >= len / 4 + 2");
    if (om && (stride % 4 || U < 4 || U > 64 || U % 4 || ngrp * (size_t)U < rowlen))
        return tetra_fail(ctx, TETRA_E_INVALID, "timing_chunks with om: stride a multiple of 4, 4 <= U <= 64 a "
                                                "multiple of 4, ngrp U >= rowlen");
    return launch_timing_chunks(ctx, P, y, M, rowlen, nchunk, stride, len, om, ngrp, U, soft, softbits, hard, nsym,
                                smax, diag);
}

int tetra_demod_etsi(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *iq, size_t C, size_t N, void *soft,
                     int8_t *softbits, uint8_t *hard, int32_t *nsym, size_t smax, float *diag) {
    return tetra_demod_etsi_fmt(ctx, P, iq, TETRA_CF32, C, N, soft, softbits, hard, nsym, smax, diag);
}

int tetra_demod_etsi_fmt(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *iq, int fmt, size_t C, size_t N,
                         void *soft, int8_t *softbits, uint8_t *hard, int32_t *nsym, size_t smax, float *diag) {
    if (!ctx) return TETRA_E_INVALID;
    int rc = etsi_check(ctx, P);
    if (rc) return rc;
    int64_t M1, M2, sm;
    tetra_etsi_lengths(P, N, &M1, &M2, &sm);
    if (M2 <= 0 || N % 2 || C == 0) return tetra_fail(ctx, TETRA_E_INVALID, "bad chunk for the ETSI demod");
    if (fmt != TETRA_CF32 && fmt != TETRA_SC16) return tetra_fail(ctx, TETRA_E_INVALID, "iq_fmt must be cf32 or sc16");
    if ((int64_t)smax < sm) return tetra_fail(ctx, TETRA_E_INVALID, "smax < %ld", (long)sm);
    Staging st(ctx);
    const void *x = st.in(iq, C * N * (fmt == TETRA_SC16 ? 4 : 8));
    void *so = st.out(soft, C * smax * 8);
    int8_t *sbo = (int8_t *)st.out(softbits, C * smax * 2);
    uint8_t *ho = (uint8_t *)st.out(hard, C * smax);
    int32_t *no = (int32_t *)st.out(nsym, C * 4);
    float *dg = diag ? (float *)st.out(diag, C * 16) : nullptr;
    if (!x || !so || !sbo || !ho || !no) return st.finish();
    // fused: timing runs in the channel filter's workgroup on y in LDS (k_chanfilt_r: y never leaves
    // LDS; k_chanfilt<uint2>: y round-trips through a C x M2 scratch and is re-staged into the freed
    // image) (measured: cf32 with y through L2 at four workgroups per CU is 2.5 % slower)
    const bool fuse = canonical(P) && fused_fits(fmt, M2, sm, N);
    if (fuse) {
        float2 *ys = nullptr;   // k_chanfilt<uint2>: y's round trip
        if (fmt == TETRA_SC16 && !per_wave(fmt, M2, N) && !(ys = (float2 *)ws(ctx, S_W3, C * (size_t)M2 * 8)))
            return st.finish();
        const TimingOut to{P->gain, P->soft_scale, (float2 *)so, sbo, ho, no, (float4 *)dg, (int)smax, timing_probe()};
        rc = launch_chanfilt(ctx, P, x, fmt, C, N, M1, M2, ys, &to);
        if (rc) return rc;
        return st.finish();
    }
    float2 *yb = (float2 *)ws(ctx, S_W3, C * (size_t)M2 * 8);
    float2 *dscr = (float2 *)ws(ctx, S_W4, C * smax * 8);
    if (!yb || !dscr) return st.finish();
    rc = launch_chanfilt(ctx, P, x, fmt, C, N, M1, M2, yb);
    if (rc) return rc;
    {
        PROF(ctx, "etsi_timing");
        hipLaunchKernelGGL(timing_kernel(M2, smax), dim3((unsigned)C), dim3(64), 0, ctx->stream, (const float2 *)yb, (int)M2, P->gain,
                           P->soft_scale, (float2 *)so, dscr, sbo, ho, no, (int)smax, (float4 *)dg, timing_probe(),
                           nullptr, 0, 0, 0, nullptr, 0, 0, 0, 0);
    }
    return st.finish();
}

int tetra_etsi_stream_window(const tetra_etsi_plan *P, int64_t x_total, int64_t y_done, int64_t n, int64_t *s,
                             int64_t *W, int64_t *yoff, int64_t *y_done_next) {
    if (!P || !s || !W || !yoff || !y_done_next || x_total < 0 || y_done < 0 || n < 0 || P->q1 < 1 || P->up < 1 ||
        P->down < 1)
        return TETRA_E_INVALID;
    // pb = q1 down input samples carry `up` outputs: a window starting at a multiple of pb has the
    // polyphase phases of a run over the whole capture, its output m is global output m + up s / pb.
    // Windows start at multiples of per = pb, doubled when odd (whole sample pairs: the kernels load
    // two samples at a time), which carry ups outputs.
    const int64_t pb = (int64_t)P->q1 * P->down, per = pb % 2 ? 2 * pb : pb, ups = P->up * (per / pb);
    int64_t st = 0;
    if (y_done > 0) {
        const int64_t a = y_done - TETRA_ETSI_MARGIN;
        st = per * (a >= 0 ? a / ups : -((-a + ups - 1) / ups));   // floor division
        if (st < 0) st = 0;
    }
    int64_t m1, m2, sm;
    tetra_etsi_lengths(P, (size_t)(x_total + n), &m1, &m2, &sm);
    *s = st;
    *W = x_total + n - st;
    *yoff = y_done - P->up * (st / pb);
    *y_done_next = m2 > y_done ? m2 : y_done;
    return TETRA_OK;
}

int tetra_demod_etsi_stream(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *iq, int fmt, size_t C, size_t ld,
                            size_t W, int yoff, tetra_etsi_track *track, void *soft, int8_t *softbits, uint8_t *hard,
                            int32_t *nsym, size_t smax, size_t ostride, float *diag) {
    if (!ctx) return TETRA_E_INVALID;
    int rc = etsi_check(ctx, P);
    if (rc) return rc;
    int64_t M1, M2, sm;
    tetra_etsi_lengths(P, W, &M1, &M2, &sm);
    if (!track || C == 0 || W % 2 || ld < W || yoff < 0 || ostride < smax)
        return tetra_fail(ctx, TETRA_E_INVALID, "demod_etsi_stream: track, W even <= ld, yoff >= 0, ostride >= smax");
    if (fmt != TETRA_CF32 && fmt != TETRA_SC16) return tetra_fail(ctx, TETRA_E_INVALID, "iq_fmt must be cf32 or sc16");
    if (fmt == TETRA_SC16 && ld % 2) return tetra_fail(ctx, TETRA_E_INVALID, "SC16 rows: ld even");
    if ((int64_t)smax < sm + 1) return tetra_fail(ctx, TETRA_E_INVALID, "smax < %ld", (long)sm + 1);
    const size_t bps = fmt == TETRA_SC16 ? 4 : 8;
    Staging st(ctx);
    tetra_etsi_track *tr = (tetra_etsi_track *)st.inout(track, C * sizeof(tetra_etsi_track));
    if (M2 <= 0) {   // a window too short for the channel filter: no outputs; the loop's position moves on
        int32_t *no = (int32_t *)st.out(nsym, C * 4);
        if (!tr || !no) return st.finish();
        HIP_TRY(ctx, hipMemsetAsync(no, 0, C * 4, ctx->stream));
        hipLaunchKernelGGL(k_track_skip, dim3(grid_for(C, 256)), dim3(256), 0, ctx->stream, tr, (int)C, yoff, (int)M2);
        return st.finish();
    }
    const void *x = st.in(iq, ((C - 1) * ld + W) * bps);
    void *so = st.out(soft, C * ostride * 8);
    int8_t *sbo = (int8_t *)st.out(softbits, C * ostride * 2);
    uint8_t *ho = (uint8_t *)st.out(hard, C * ostride);
    int32_t *no = (int32_t *)st.out(nsym, C * 4);
    float *dg = diag ? (float *)st.out(diag, C * 16) : nullptr;
    if (!tr || !x || !so || !sbo || !ho || !no) return st.finish();
    // SC16's per-wave kernel loads 16-B groups of 4 samples: rows (ld) and the window (W) in whole groups
    const size_t Wk = (fmt == TETRA_SC16 && ld % 4) ? W + 1 : W;   // (an odd row pitch: not per-wave)
    const bool fuse = canonical(P) && fused_fits(fmt, M2, sm + 1, Wk);
    if (fuse) {
        float2 *ys = nullptr;
        if (fmt == TETRA_SC16 && !per_wave(fmt, M2, Wk) && !(ys = (float2 *)ws(ctx, S_W3, C * (size_t)M2 * 8)))
            return st.finish();
        TimingOut to{P->gain, P->soft_scale, (float2 *)so, sbo, ho, no, (float4 *)dg, (int)smax, timing_probe()};
        to.ostride = (int)ostride;
        to.yoff = yoff;
        to.track = tr;
        rc = launch_chanfilt(ctx, P, x, fmt, C, W, M1, M2, ys, &to, ld, Wk);
        if (rc) return rc;
        return st.finish();
    }
    float2 *yb = (float2 *)ws(ctx, S_W3, C * (size_t)M2 * 8);
    float2 *dscr = (float2 *)ws(ctx, S_W4, C * smax * 8);
    if (!yb || !dscr) return st.finish();
    rc = launch_chanfilt(ctx, P, x, fmt, C, W, M1, M2, yb, nullptr, ld, Wk);
    if (rc) return rc;
    {
        PROF(ctx, "etsi_timing");
        hipLaunchKernelGGL(timing_kernel(M2, smax), dim3((unsigned)C), dim3(64), 0, ctx->stream, (const float2 *)yb,
                           (int)M2, P->gain, P->soft_scale, (float2 *)so, dscr, sbo, ho, no, (int)smax, (float4 *)dg,
                           timing_probe(), nullptr, 0, 0, 0, tr, yoff, (int)ostride, 0, 0);
    }
    return st.finish();
}


int tetra_etsi_decide(tetra_ctx *ctx, const void *x, int fmt, size_t n, uint8_t *hard) {
    if (!ctx || (fmt != TETRA_CF32 && fmt != TETRA_CF64)) return TETRA_E_INVALID;
    if (n < 2) return TETRA_OK;
    Staging st(ctx);
    const void *xd = st.in(x, n * (fmt == TETRA_CF64 ? 16 : 8));
    uint8_t *h = (uint8_t *)st.out(hard, n - 1);
    if (!xd || !h) return st.finish();
    if (fmt == TETRA_CF32)
        hipLaunchKernelGGL(k_etsi_decide<float2>, dim3(grid_for(n - 1, 256)), dim3(256), 0, ctx->stream,
                           (const float2 *)xd, (long)n, h);
    else
        hipLaunchKernelGGL(k_etsi_decide<double2>, dim3(grid_for(n - 1, 256)), dim3(256), 0, ctx->stream,
                           (const double2 *)xd, (long)n, h);
    return st.finish();
}

int tetra_etsi_decode_blocks(tetra_ctx *ctx, const int8_t *soft5, size_t F, int kind, const uint32_t *scramb_init,
                             uint8_t *type1, uint8_t *crc_ok) {
    if (!ctx || kind < 0 || kind > 2) return TETRA_E_INVALID;
    if (F == 0) return TETRA_OK;
    const KindP P = kind_params(kind);
    std::vector<uint32_t> init(F);
    HIP_TRY(ctx, hipMemcpy(init.data(), scramb_init, F * 4, hipMemcpyDefault));
    std::vector<uint8_t> tab(F * P.K);
    for (size_t f = 0; f < F; ++f) scramble_seq(init[f], P.K, tab.data() + f * P.K);
    Staging st(ctx);
    const int8_t *s = (const int8_t *)st.in(soft5, F * P.K);
    const uint8_t *scr = (const uint8_t *)st.in(tab.data(), tab.size());
    uint8_t *t = (uint8_t *)st.out(type1, F * P.n1);
    uint8_t *o = (uint8_t *)st.out(crc_ok, F);
    if (!s || !scr || !t || !o) return st.finish();
    {
        PROF(ctx, "etsi_decode_blocks");
        hipLaunchKernelGGL(k_decode_blocks, dim3((unsigned)((F + 3) / 4)), dim3(64), 0, ctx->stream, s, (int)F, kind,
                           scr, t, o);
    }
    return st.finish();
}

int tetra_etsi_encode_blocks(tetra_ctx *ctx, const uint8_t *type1, size_t F, int kind, const uint32_t *scramb_init,
                             uint8_t *type5) {
    if (!ctx || kind < 0 || kind > 2) return TETRA_E_INVALID;
    if (F == 0) return TETRA_OK;
    const KindP P = kind_params(kind);
    std::vector<uint32_t> init(F);
    HIP_TRY(ctx, hipMemcpy(init.data(), scramb_init, F * 4, hipMemcpyDefault));
    std::vector<uint8_t> tab(F * P.K);
    for (size_t f = 0; f < F; ++f) scramble_seq(init[f], P.K, tab.data() + f * P.K);
    Staging st(ctx);
    const uint8_t *t = (const uint8_t *)st.in(type1, F * P.n1);
    const uint8_t *scr = (const uint8_t *)st.in(tab.data(), tab.size());
    uint8_t *o = (uint8_t *)st.out(type5, F * P.K);
    if (!t || !scr || !o) return st.finish();
    hipLaunchKernelGGL(k_encode_blocks, dim3((unsigned)((F + 63) / 64)), dim3(64), 0, ctx->stream, t, (int)F, kind, scr,
                       o);
    return st.finish();
}

// The lower MAC's launch sequence; cell_init (device) selects acquisition, else the configured cells.
static int lmac_etsi(tetra_ctx *ctx, const int8_t *softbits, const uint8_t *hard, const int32_t *nsym, size_t C,
                     size_t smax, uint32_t *cell_init, int32_t *nburst, int32_t *bursts, int32_t *nblock,
                     int32_t *blocks, uint8_t *type1, int32_t *lead = nullptr, int8_t *next_soft = nullptr,
                     uint8_t *next_hard = nullptr) {
    if (!ctx || C == 0) return TETRA_E_INVALID;
    if (!cell_init && ctx->cells < C)
        return tetra_fail(ctx, TETRA_E_INVALID, "tetra_etsi_set_cells() for %zu channels first", C);
    if (2 * smax > LMAC_MAXBITS + 4) return tetra_fail(ctx, TETRA_E_INVALID, "chunk too long for tetra_lmac_etsi");
    // k_etsi_viterbi reads the soft bits and the cell table through 32-bit buffer offsets
    if (C * smax * 2 + 8 > (size_t)INT32_MAX || (C + 1) * 432 > (size_t)INT32_MAX)
        return tetra_fail(ctx, TETRA_E_INVALID, "too many channels for one tetra_lmac_etsi call (%zu)", C);
    Staging st(ctx);
    uint32_t *ci = cell_init ? (uint32_t *)st.inout(cell_init, C * 4) : nullptr;
    // streaming into the input rows themselves: host rows are staged in and back out (with the tail)
    const bool alias = lead && next_soft == softbits;
    const int8_t *sb = alias ? (const int8_t *)st.inout(const_cast<int8_t *>(softbits), C * smax * 2)
                             : (const int8_t *)st.in(softbits, C * smax * 2);
    const uint8_t *hd = alias ? (const uint8_t *)st.inout(const_cast<uint8_t *>(hard), C * smax)
                              : (const uint8_t *)st.in(hard, C * smax);
    // streaming: the scan state and the rows the tail goes to
    int32_t *ld_ = lead ? (int32_t *)st.inout(lead, C * 4) : nullptr;
    int8_t *nsb = nullptr;
    uint8_t *nhd = nullptr;
    if (lead) {
        nsb = next_soft == softbits ? const_cast<int8_t *>(sb) : (int8_t *)st.inout(next_soft, C * smax * 2);
        nhd = next_hard == hard ? const_cast<uint8_t *>(hd) : (uint8_t *)st.inout(next_hard, C * smax);
        if (!ld_ || !nsb || !nhd) return st.finish();
    }
    const int32_t *ns = (const int32_t *)st.in(nsym, C * 4);
    int32_t *nbo = (int32_t *)st.out(nburst, C * 4);
    int32_t *bo = (int32_t *)st.out(bursts, C * ETSI_MAXB * 2 * 4);
    int32_t *nko = (int32_t *)st.out(nblock, C * 4);
    int32_t *ko = (int32_t *)st.out(blocks, C * ETSI_MAXJ * 4 * 4);
    uint8_t *to = (uint8_t *)st.out(type1, C * ETSI_MAXJ * 268);
    const size_t jtot = 32 * C;   // the three job regions (job_base / job_cap)
    // workspace: [job counters per kind (16 B)] [jobs] [survivors: 36 groups x jtot x 4 lanes x 32 bits
    // (SCH/F: 288 steps / 8; allocated as 288 x jtot dwords)]
    char *w = (char *)ws(ctx, S_W7, 16 + jtot * sizeof(Job) + 288 * jtot * 4 + (lead ? 8 * C : 0));
    if ((cell_init && !ci) || !sb || !hd || !ns || !nbo || !bo || !nko || !ko || !to || !w) return st.finish();
    unsigned long long *jcount = (unsigned long long *)w;
    Job *jobs = (Job *)(w + 16);
    uint32_t *surv = (uint32_t *)(w + 16 + jtot * sizeof(Job));
    int32_t *tinfo = lead ? (int32_t *)(w + 16 + jtot * sizeof(Job) + 288 * jtot * 4) : nullptr;   // streaming
    if (cell_init && ctx->cells != C) {   // acquisition on a new channel count: an empty table
        std::vector<uint8_t> bsch(432);
        scramble_seq(3u, 432, bsch.data());
        uint8_t *tab = (uint8_t *)ws(ctx, S_W5, C * 432 + 432);
        uint32_t *ti = (uint32_t *)ws(ctx, S_W14, C * 4);
        if (!tab || !ti) return TETRA_E_NOMEM;
        HIP_TRY(ctx, hipMemcpyAsync(tab + C * 432, bsch.data(), 432, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(ti, 0, C * 4, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));   // bsch is a pageable host buffer
        ctx->cells = C;
    }
    uint8_t *cells = (uint8_t *)ctx->slot[S_W5].p;
    const uint8_t *bsch_scr = cells + ctx->cells * 432;
    {
        PROF(ctx, "etsi_sync");
        HIP_TRY(ctx, hipMemsetAsync(jcount, 0, 16, ctx->stream));
        const unsigned ngrp = (unsigned)((C + SYNC_WAVES - 1) / SYNC_WAVES);
        // double-buffered rows: the sync kernel moves the tails itself (no k_etsi_tail launch)
        const bool other = lead && nhd != hd;
        hipLaunchKernelGGL(k_etsi_sync, dim3(ngrp), dim3(64 * SYNC_WAVES), 0,
                           ctx->stream, hd, ns, (int)smax, nbo, bo, nko, jcount, jobs, (int)C, ld_,
                           lead ? TETRA_ETSI_RESERVE : 0, tinfo, sb, other ? nhd : nullptr, other ? nsb : nullptr);
    }
    // grids: the waves each kind's job capacity needs (16 blocks per trellis wave, 64 per traceback wave)
    // (TETRA_LMAC_GRID_CAP: at most that many trellis workgroups, a quarter as many traceback ones --
    // the kernels walk their jobs with a grid stride; 0 = the capacity)
    static const long gcap = getenv("TETRA_LMAC_GRID_CAP") ? atol(getenv("TETRA_LMAC_GRID_CAP")) : 0;
    auto vgrid = [&](int m) {
        size_t g = 0;
        for (int k = 0; k < 3; ++k) g += (m >> k) & 1 ? (job_cap(k, C) + 15) / 16 : 0;
        if (gcap > 0 && g > (size_t)gcap) g = (size_t)gcap;
        return dim3((unsigned)g);
    };
    auto tgrid = [&](int m) {
        size_t g = 0;
        for (int k = 0; k < 3; ++k) g += (m >> k) & 1 ? (job_cap(k, C) + 63) / 64 : 0;
        if (gcap > 0 && g > (size_t)(gcap / 4 + 1)) g = (size_t)(gcap / 4 + 1);
        return dim3((unsigned)g);
    };
    int mask = 7;
    if (ci) {   // BSCH first (colour code 0), then the cell from it, then SCH/F + SCH/HD
        PROF(ctx, "etsi_acquire");
        hipLaunchKernelGGL(k_etsi_viterbi, vgrid(4), dim3(64), 0, ctx->stream, jobs, jcount, (int)C, sb, (int)smax,
                           cells, bsch_scr, surv, 4);
        hipLaunchKernelGGL(k_etsi_traceback, tgrid(4), dim3(64), 0, ctx->stream, jobs, jcount, (int)C, surv, ko, to, 4);
        hipLaunchKernelGGL(k_cell_acquire, dim3(grid_for(C, 256)), dim3(256), 0, ctx->stream, (int)C, nbo, bo, ko, to,
                           ci, (uint32_t *)ctx->slot[S_W14].p, cells);
        mask = 3;
    }
    {
        PROF(ctx, "etsi_viterbi");
        hipLaunchKernelGGL(k_etsi_viterbi, vgrid(mask), dim3(64), 0, ctx->stream, jobs, jcount, (int)C, sb, (int)smax,
                           cells, bsch_scr, surv, mask);
    }
    {
        PROF(ctx, "etsi_traceback");
        hipLaunchKernelGGL(k_etsi_traceback, tgrid(mask), dim3(64), 0, ctx->stream, jobs, jcount, (int)C, surv, ko, to,
                           mask);
    }
    if (lead && nhd == hd) {   // these rows: the tails after the trellis has read them
        PROF(ctx, "etsi_tail");
        hipLaunchKernelGGL(k_etsi_tail, dim3((unsigned)C), dim3(64), 0, ctx->stream, hd, sb, (int)smax, (int)C, tinfo,
                           TETRA_ETSI_RESERVE, nhd, nsb, ld_);
    }
    return st.finish();
}

int tetra_lmac_etsi(tetra_ctx *ctx, const int8_t *softbits, const uint8_t *hard, const int32_t *nsym, size_t C,
                    size_t smax, int32_t *nburst, int32_t *bursts, int32_t *nblock, int32_t *blocks, uint8_t *type1) {
    return lmac_etsi(ctx, softbits, hard, nsym, C, smax, nullptr, nburst, bursts, nblock, blocks, type1);
}

int tetra_lmac_etsi_acquire(tetra_ctx *ctx, const int8_t *softbits, const uint8_t *hard, const int32_t *nsym,
                            size_t C, size_t smax, uint32_t *cell_init, int32_t *nburst, int32_t *bursts,
                            int32_t *nblock, int32_t *blocks, uint8_t *type1) {
    if (!cell_init) return tetra_fail(ctx, TETRA_E_INVALID, "cell_init is NULL");
    return lmac_etsi(ctx, softbits, hard, nsym, C, smax, cell_init, nburst, bursts, nblock, blocks, type1);
}

int tetra_lmac_etsi_stream(tetra_ctx *ctx, const int8_t *softbits, const uint8_t *hard, const int32_t *nsym,
                           size_t C, size_t stride, int32_t *lead, int8_t *next_soft, uint8_t *next_hard,
                           uint32_t *cell_init, int32_t *nburst, int32_t *bursts, int32_t *nblock, int32_t *blocks,
                           uint8_t *type1) {
    if (!lead || !next_soft || !next_hard || stride <= TETRA_ETSI_RESERVE)
        return tetra_fail(ctx, TETRA_E_INVALID, "lmac_etsi_stream: lead, next rows and stride > TETRA_ETSI_RESERVE");
    if ((next_soft == softbits) != (next_hard == hard))
        return tetra_fail(ctx, TETRA_E_INVALID, "lmac_etsi_stream: next rows must both alias the inputs or neither");
    return lmac_etsi(ctx, softbits, hard, nsym, C, stride, cell_init, nburst, bursts, nblock, blocks, type1, lead,
                     next_soft, next_hard);
}

}  // extern "C"
