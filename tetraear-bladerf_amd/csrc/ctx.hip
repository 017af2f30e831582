// ctx.hip -- context lifecycle, error reporting and host/device argument staging.
#include "common.h"

thread_local std::string g_tetra_err;

int tetra_fail(tetra_ctx *ctx, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    g_tetra_err = buf;
    return code;
}

void *ws(tetra_ctx *ctx, int s, size_t bytes) {
    DevBuf &b = ctx->slot[s];
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return b.p;
    if (s == S_W16) ctx->sosb_valid = false;   // the uploaded Phi table lives in this slot
    if (b.p) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
    }
    size_t want = bytes + (bytes >> 3);   // headroom against regrowth
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        tetra_fail(ctx, TETRA_E_NOMEM, "hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
        b.p = nullptr;
        return nullptr;
    }
    b.bytes = want;
    return b.p;
}

bool is_device_ptr(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

void *Staging::pin_take(size_t bytes) {
    if (bytes > PIN_SMALL) return nullptr;
    if (!ctx->pin) {
        if (hipHostMalloc(&ctx->pin, PIN_ARENA) != hipSuccess) {
            (void)hipGetLastError();
            ctx->pin = nullptr;
            return nullptr;
        }
        ctx->pin_cap = PIN_ARENA;
    }
    const size_t at = (pin_off + 255) & ~(size_t)255;
    if (at + bytes > ctx->pin_cap) return nullptr;
    pin_off = at + bytes;
    ctx->pin_busy = true;
    return (char *)ctx->pin + at;
}

const void *Staging::in(const void *p, size_t bytes) {
    if (failed) return nullptr;
    if (bytes == 0) return p ? p : ws(ctx, next_in++, 16);
    if (is_device_ptr(p)) return p;
    host_touched = true;
    if (next_in > S_IN5) {
        failed = true;
        tetra_fail(ctx, TETRA_E_INVALID, "more than %d staged host inputs", S_IN5 - S_IN0 + 1);
        return nullptr;
    }
    void *d = ws(ctx, next_in++, bytes);
    void *h = d ? pin_take(bytes) : nullptr;
    if (h) memcpy(h, p, bytes);
    if (!d || hipMemcpyAsync(d, h ? h : p, bytes, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) {
        failed = true;
        if (d) tetra_fail(ctx, TETRA_E_HIP, "H2D staging copy failed");
        return nullptr;
    }
    return d;
}

void *Staging::out(void *p, size_t bytes) {
    if (failed) return nullptr;
    if (bytes == 0) return p ? p : ws(ctx, next_out++, 16);
    if (is_device_ptr(p)) return p;
    host_touched = true;
    if (next_out > S_OUT9) {   // never into the kernels' workspace slots
        failed = true;
        tetra_fail(ctx, TETRA_E_INVALID, "more than %d staged host outputs", S_OUT9 - S_OUT0 + 1);
        return nullptr;
    }
    void *d = ws(ctx, next_out++, bytes);
    if (!d) {
        failed = true;
        return nullptr;
    }
    back.push_back({p, d, bytes, pin_take(bytes)});
    return d;
}

void *Staging::inout(void *p, size_t bytes) {
    if (failed) return nullptr;
    if (is_device_ptr(p)) return p;
    void *d = out(p, bytes);
    if (d && hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) {
        failed = true;
        tetra_fail(ctx, TETRA_E_HIP, "H2D staging copy failed");
        return nullptr;
    }
    return d;
}

int Staging::finish() {
    if (failed) return ctx->err.empty() ? tetra_fail(ctx, TETRA_E_HIP, "staging failed") : TETRA_E_HIP;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return tetra_fail(ctx, TETRA_E_HIP, "kernel launch failed: %s", hipGetErrorString(e));
    for (auto &b : back)
        HIP_TRY(ctx, hipMemcpyAsync(b.pin ? b.pin : b.host, b.dev, b.bytes, hipMemcpyDeviceToHost, ctx->stream));
    if (host_touched || ctx->pin_busy) HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (auto &b : back)
        if (b.pin) memcpy(b.host, b.pin, b.bytes);
    ctx->pin_busy = false;
    return TETRA_OK;
}

static hipEvent_t take_event(tetra_ctx *c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

ProfScope::ProfScope(tetra_ctx *ctx, const char *n) : c(ctx), name(n) {
    if (c && c->prof) {
        a = take_event(c);
        if (a) (void)hipEventRecord(a, c->stream);
    }
}

ProfScope::~ProfScope() {
    if (!a) return;
    hipEvent_t b = take_event(c);
    if (!b) return;
    (void)hipEventRecord(b, c->stream);
    c->recs.push_back({name, a, b});
}

extern "C" {

int tetra_profile(tetra_ctx *ctx, int enable) {
    if (!ctx) return TETRA_E_INVALID;
    ctx->prof = enable != 0;
    return TETRA_OK;
}

int tetra_profile_read(tetra_ctx *ctx, char *names, size_t names_len, double *ms, int64_t *count, int max_stages,
                       int *n_stages) {
    if (!ctx || !n_stages) return TETRA_E_INVALID;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<std::string> nm;
    std::vector<double> acc;
    std::vector<int64_t> cnt;
    for (auto &r : ctx->recs) {
        float t = 0.f;
        (void)hipEventElapsedTime(&t, r.a, r.b);
        size_t i = 0;
        while (i < nm.size() && nm[i] != r.name) ++i;
        if (i == nm.size()) { nm.push_back(r.name); acc.push_back(0); cnt.push_back(0); }
        acc[i] += t;
        cnt[i] += 1;
        ctx->ev_pool.push_back(r.a);
        ctx->ev_pool.push_back(r.b);
    }
    ctx->recs.clear();
    size_t off = 0;
    int n = 0;
    for (size_t i = 0; i < nm.size() && n < max_stages; ++i, ++n) {
        if (ms) ms[n] = acc[i];
        if (count) count[n] = cnt[i];
        if (names && off + nm[i].size() + 1 < names_len) {
            memcpy(names + off, nm[i].c_str(), nm[i].size() + 1);
            off += nm[i].size() + 1;
        }
    }
    if (names && off < names_len) names[off] = 0;
    *n_stages = n;
    return TETRA_OK;
}

int tetra_abi_version(void) { return TETRA_ABI_VERSION; }

tetra_ctx *tetra_create(int device) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        tetra_fail(nullptr, TETRA_E_NODEVICE, "no HIP device visible (%s)", hipGetErrorString(e));
        return nullptr;
    }
    if (device < 0 || device >= n) {
        tetra_fail(nullptr, TETRA_E_INVALID, "device %d out of range (%d devices)", device, n);
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || hipSetDevice(device) != hipSuccess) {
        tetra_fail(nullptr, TETRA_E_HIP, "cannot open device %d", device);
        return nullptr;
    }
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        tetra_fail(nullptr, TETRA_E_NODEVICE, "device %d is %s; libtetra_hip is built for gfx950", device,
                   prop.gcnArchName);
        return nullptr;
    }
    tetra_ctx *ctx = new tetra_ctx();
    ctx->device = device;
    snprintf(ctx->arch, sizeof ctx->arch, "%s", prop.gcnArchName);
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        tetra_fail(nullptr, TETRA_E_HIP, "hipStreamCreate failed");
        delete ctx;
        return nullptr;
    }
    return ctx;
}

void tetra_destroy(tetra_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto &r : ctx->recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    for (auto e : ctx->ev_pool) (void)hipEventDestroy(e);
    if (ctx->fft && ctx->fft_free) ctx->fft_free(ctx->fft);
    for (auto &b : ctx->slot)
        if (b.p) (void)hipFree(b.p);
    if (ctx->pin) (void)hipHostFree(ctx->pin);
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *tetra_last_error(const tetra_ctx *ctx) { return ctx ? ctx->err.c_str() : g_tetra_err.c_str(); }

void *tetra_get_stream(tetra_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int tetra_set_stream(tetra_ctx *ctx, void *s) {
    if (!ctx) return TETRA_E_INVALID;
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    ctx->stream = (hipStream_t)s;
    ctx->own_stream = false;
    return TETRA_OK;
}

int tetra_synchronize(tetra_ctx *ctx) {
    if (!ctx) return TETRA_E_INVALID;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return TETRA_OK;
}

int tetra_device_arch(tetra_ctx *ctx, char *buf, size_t n) {
    if (!ctx || !buf || !n) return TETRA_E_INVALID;
    snprintf(buf, n, "%s", ctx->arch);
    return TETRA_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ HBM read floor (diagnostic)
// The access pattern of the channel filter without its arithmetic: one workgroup streams one row
// of `row_bytes` with 16-B nontemporal loads (the load form the channel filter uses), two groups of
// five per thread in flight (a register ring, like the filter's two-tile prefetch), folded into one
// word so nothing is dead-code eliminated.  `lds_bytes` of dynamic LDS caps the workgroups per CU
// the way the real kernel's LDS does.  bench.py reports it as the measured floor beside the
// roofline.  (tools/probes/probe_hbm.hip: plain loads 6.15-6.19 TB/s, nt 6.91-7.07 TB/s.)
__global__ __launch_bounds__(256) void k_read_floor(const float4 *__restrict__ x, long row4, uint32_t *out) {
    extern __shared__ float4 pad_lds[];
    const float4 *p = x + (size_t)blockIdx.x * row4;
    uint32_t acc = 0;
    float4 v[2][5];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int r = 0; r < 5; ++r) v[d][r] = ld_nt(p + min((long)(d * 5 + r) * 256 + threadIdx.x, row4 - 1));
    for (long g = 0; g * 1280 < row4; g += 2) {
#pragma unroll
        for (int d = 0; d < 2; ++d) {
#pragma unroll
            for (int r = 0; r < 5; ++r)
                acc ^= __float_as_uint(v[d][r].x) ^ __float_as_uint(v[d][r].y) ^ __float_as_uint(v[d][r].z) ^
                       __float_as_uint(v[d][r].w);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int r = 0; r < 5; ++r) v[d][r] = ld_nt(p + min((g + 2 + d) * 1280 + r * 256 + threadIdx.x, row4 - 1));
        }
    }
    if (acc == 0x9E3779B9u) pad_lds[threadIdx.x] = make_float4(0.f, 0.f, 0.f, 0.f);   // keeps the LDS allocation
    if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;   // practically never: no store traffic
}

extern "C" int tetra_read_floor(tetra_ctx *ctx, const void *x, size_t rows, size_t row_bytes, size_t lds_bytes) {
    if (!ctx || !x || rows == 0 || row_bytes % 16 || lds_bytes > 160 * 1024) return TETRA_E_INVALID;
    uint32_t *o = (uint32_t *)ws(ctx, S_W13, rows * 4);
    if (!o) return TETRA_E_NOMEM;
    PROF(ctx, "read_floor");
    hipLaunchKernelGGL(k_read_floor, dim3((unsigned)rows), dim3(256), lds_bytes, ctx->stream, (const float4 *)x,
                       (long)(row_bytes / 16), o);
    HIP_TRY(ctx, hipGetLastError());
    return TETRA_OK;
}

// ------------------------------------------------------------------ profile region marker (diagnostic)
// One 64-lane wave that stores `tag` into the diagnostics slot (a vector store by lane 0).  bench.py
// launches it on the context stream right before and right after its timed steps, so a rocprofv3
// kernel trace or counter collection of the bench command can pick out the timed launches by
// dispatch order (tools/pmc_summary.py: the launches between the two k_region_mark dispatches).
__global__ __launch_bounds__(64) void k_region_mark(int tag, int *out) {
    if (threadIdx.x == 0) out[0] = tag;
}

extern "C" int tetra_mark(tetra_ctx *ctx, int tag) {
    if (!ctx) return TETRA_E_INVALID;
    int *o = (int *)ws(ctx, S_W13, 256);
    if (!o) return TETRA_E_NOMEM;
    hipLaunchKernelGGL(k_region_mark, dim3(1), dim3(64), 0, ctx->stream, tag, o);
    HIP_TRY(ctx, hipGetLastError());
    return TETRA_OK;
}
