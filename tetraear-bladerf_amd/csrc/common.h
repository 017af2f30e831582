// common.h -- shared plumbing for libtetra_hip.so (context, errors, host/device staging).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <type_traits>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tetra_hip.h"

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

// Workspace slots owned by a context (grown on demand, never shrunk).
enum Slot {
    S_IN0 = 0, S_IN1, S_IN2, S_IN3, S_IN4, S_IN5,          // staged host inputs
    S_OUT0, S_OUT1, S_OUT2, S_OUT3, S_OUT4, S_OUT5,        // staged host outputs
    S_OUT6, S_OUT7, S_OUT8, S_OUT9,                        // (the streaming lower MAC stages nine)
    S_W0, S_W1, S_W2, S_W3, S_W4, S_W5, S_W6, S_W7,        // kernel workspaces
    S_W8, S_W9, S_W10,                                     // wideband channeliser
    S_W11,                                                 // waterfall window + twiddles
    S_W12,                                                 // ETSI channel-filter tap image (kept)
    S_W13,                                                 // diagnostics (tetra_read_floor sink)
    S_W14,                                                 // ETSI: scrambler inits the cell table holds
    S_W15,                                                 // ETSI generic-rate tap tables (etsi_rate.hip)
    S_W16,                                                 // compat time-blocked decimator: tile states, Phi table
    S_W17,                                                 // compat time-blocked filtfilt: tile states
    S_W18,                                                 // compat latency mode: extract_symbols' |y|^2 rows
    S_W19,                                                 // compat, few channels: the mixed rows filtfilt reads
    S_COUNT
};

struct ProfRec {
    const char *name;
    hipEvent_t a, b;
};

struct tetra_ctx {
    bool prof = false;                 // per-stage HIP-event timing (tetra_profile)
    std::vector<ProfRec> recs;
    std::vector<hipEvent_t> ev_pool;
    size_t cells = 0;                  // channels configured by tetra_etsi_set_cells
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;
    std::string err;
    DevBuf slot[S_COUNT];
    char arch[64] = {0};
    float coef_etsi[128 + 39 * 64];    // host image of the channel-filter tap tables (h1, h1 / 32768, stage-2 MFMA A)
    const void *coef_etsi_dev = nullptr;   // workspace the tap image was last uploaded to
    std::vector<float> taps_rate;      // generic-rate ETSI taps (h1, hp) as last uploaded to slot S_W15
    const void *taps_rate_dev = nullptr;
    std::vector<float> taps_wb;        // host image of the wideband prototype + resampler taps
    std::vector<float> taps_wb_up;     // ... as last uploaded to taps_wb_dev (slot S_W9)
    const void *taps_wb_dev = nullptr;
    void *fft = nullptr;               // rocFFT plan cache (wideband.hip), freed by fft_free
    void (*fft_free)(void *) = nullptr;
    bool wf_tables_ready = false;      // waterfall tables uploaded to slot S_W11
    std::vector<double> sosb_tab;      // compat time-blocked decimator: Phi^(2^r) table as last uploaded
    double sosb_coef[24] = {0};        // ... built from these SOS rows (the plan is a public struct:
    bool sosb_valid = false;           //     the same q may come with other coefficients)
    const void *sosb_dev = nullptr;    // ... to this address (slot S_W16; cleared when ws() reallocates it)
    void *pin = nullptr;               // pinned host arena: small staged copies go through it (Staging)
    size_t pin_cap = 0;
    bool pin_busy = false;             // a copy through the arena may still be in flight
};

extern thread_local std::string g_tetra_err;

int tetra_fail(tetra_ctx *ctx, int code, const char *fmt, ...);

#define HIP_TRY(ctx, expr)                                                                         \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return tetra_fail((ctx), TETRA_E_HIP, "%s failed: %s (%s:%d)", #expr,                   \
                              hipGetErrorString(e_), __FILE__, __LINE__);                          \
    } while (0)

// Returns device-side workspace of >= bytes in slot s (nullptr on failure, error set).
void *ws(tetra_ctx *ctx, int s, size_t bytes);
bool is_device_ptr(const void *p);

// Host/device argument staging.  `in` returns a device pointer holding the bytes of p;
// `out` returns a device pointer whose contents are copied back to p by finish().
// Host arguments of up to PIN_SMALL bytes are staged through the context's pinned arena (an async
// copy, and one memcpy on the host), larger ones copied from/to the caller's pageable memory.
constexpr size_t PIN_SMALL = 128 << 10, PIN_ARENA = 1 << 20;
struct Staging {
    tetra_ctx *ctx;
    int next_in = S_IN0, next_out = S_OUT0;
    struct Back { void *host; const void *dev; size_t bytes; void *pin; };
    std::vector<Back> back;
    size_t pin_off = 0;
    bool host_touched = false;
    bool failed = false;
    explicit Staging(tetra_ctx *c) : ctx(c) {
        if (ctx && ctx->pin_busy) {   // an earlier call left the arena (an error path skipped finish)
            (void)hipStreamSynchronize(ctx->stream);
            ctx->pin_busy = false;
        }
    }
    void *pin_take(size_t bytes);   // 256-B aligned arena space, nullptr if none
    const void *in(const void *p, size_t bytes);
    void *out(void *p, size_t bytes);
    void *inout(void *p, size_t bytes);   // `in` + `out` on one buffer (host contents uploaded first)
    int finish();   // D2H copies (if any) + stream sync when host memory was involved
};

// Brackets the kernels launched in its scope with HIP events on the context stream when
// profiling is on: the device time of each named stage, measured on the stream it runs on.
struct ProfScope {
    tetra_ctx *c;
    const char *name;
    hipEvent_t a = nullptr;
    ProfScope(tetra_ctx *ctx, const char *n);
    ~ProfScope();
};
#define PROF_CAT2(a, b) a##b
#define PROF_CAT(a, b) PROF_CAT2(a, b)
#define PROF(ctx, name) ProfScope PROF_CAT(prof_scope_, __LINE__)((ctx), (name))

// Batched complex-to-complex rocFFT on the context stream (fft.hip): `inverse` = e^{+i}, unnormalised
// both ways; `dbl` = double precision; plans cached per context.
int fft_c2c(tetra_ctx *ctx, bool inverse, bool dbl, size_t len, size_t batch, size_t istride, size_t idist,
            size_t ostride, size_t odist, void *in, void *out);

static inline unsigned grid_for(size_t threads, unsigned block) {
    return (unsigned)((threads + block - 1) / block);
}

// Streamed-once input loads with the nontemporal hint (global_load_dwordx4 ... nt).  Measured on
// MI355X (tools/probes/probe_hbm.hip: 8192 rows x 1 MiB, one 256-thread workgroup per row):
// 6.15-6.19 TB/s with plain 16-B loads, 6.91-7.07 TB/s with nt, at every depth and occupancy tried.
typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef unsigned nt_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 ld_nt(const float4 *p) {
    const nt_f4 v = __builtin_nontemporal_load(reinterpret_cast<const nt_f4 *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ld_nt(const uint2 *p) {
    const nt_u2 v = __builtin_nontemporal_load(reinterpret_cast<const nt_u2 *>(p));
    return make_uint2(v.x, v.y);
}

// ETSI channel filter at a non-canonical rate (etsi_rate.hip): plan limits (nullptr = supported),
// the launch (y [C][M2] to HBM), and the kernel symbol (tetra_etsi_kernel_info).
const char *etsi_generic_unsupported(const tetra_etsi_plan *P);
int launch_chanfilt_generic(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *x, int fmt, size_t C, size_t N,
                            int64_t M1, int64_t M2, float2 *y, size_t ld = 0);   // ld: row pitch (0: N)
const void *chanfilt_generic_fn(int fmt);
