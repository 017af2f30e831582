// fft.hip -- rocFFT plumbing (plan cache per context) and the FFT resampler behind
// SignalProcessor.resample (/root/reference/tetraear/signal/processor.py:35-49), which calls
// scipy.signal.resample(samples, int(len * target / fs)).  For complex input that is (scipy 1.15.3
// signal/_signaltools.py resample, domain='time', no window):
//   X = fft(x)                                   length Nx
//   Y[0 : N/2+1] = X[0 : N/2+1],  Y[num-(N-N/2-1) :] = X[Nx-(N-N/2-1) :]   with N = min(num, Nx)
//   N even, num < Nx (down):  Y[num - N/2] += X[Nx - N/2]     (the two Nyquist halves joined)
//   N even, num > Nx (up):    Y[N/2] *= 1/2, Y[num - N/2] = Y[N/2]   (the Nyquist bin split)
//   y = ifft(Y) * num / Nx                       length num
// Here: forward rocFFT (in the input's precision), one kernel that builds Y with the 1/Nx scale
// folded in, unnormalised inverse rocFFT.  Parity is a tolerance against scipy (tests/test_resample.py).
#include "common.h"

#include <rocfft/rocfft.h>

#include <mutex>

namespace {

struct FftPlan {
    bool inverse, dbl;
    size_t len, batch, istride, idist, ostride, odist;
    bool inplace;
    rocfft_plan plan;
    rocfft_execution_info info;
    size_t work;
};
struct FftCache {
    std::vector<FftPlan> plans;
    DevBuf work;
};
constexpr size_t FFT_MAX_PLANS = 24;   // arbitrary-length resample calls would grow the cache otherwise

void destroy_plan(FftPlan &f) {
    rocfft_execution_info_destroy(f.info);
    rocfft_plan_destroy(f.plan);
}

void fft_free(void *p) {
    auto *c = static_cast<FftCache *>(p);
    for (auto &f : c->plans) destroy_plan(f);
    if (c->work.p) (void)hipFree(c->work.p);
    delete c;
}

std::once_flag g_fft_once;

template <typename T2, typename T>
__global__ __launch_bounds__(256) void k_resample_spectrum(const T2 *__restrict__ X, long Nx, long num, T scale,
                                                           T2 *__restrict__ Y) {
    const long k = (long)blockIdx.x * 256 + threadIdx.x;
    const long c = blockIdx.y;
    if (k >= num) return;
    const T2 *x = X + c * Nx;
    const long N = num < Nx ? num : Nx, nyq = N / 2 + 1, neg = N - nyq;   // neg: negative-frequency bins kept
    T2 v;
    v.x = 0;
    v.y = 0;
    if (k < nyq) {
        v = x[k];
    } else if (N > 2 && k >= num - neg) {
        v = x[Nx - (num - k)];
    }
    if (N % 2 == 0) {
        const long h = N / 2;
        // (scipy's slice(-N//2, -N//2 + 1) is empty for N = 2: no join there)
        if (num < Nx && N > 2 && k == num - h) {   // downsampling: Y[-N/2] += X[-N/2] (the +N/2 bin when num = N)
            const T2 a = x[Nx - h];
            v.x += a.x;
            v.y += a.y;
        } else if (num > Nx && (k == h || k == num - h)) {   // upsampling: split the Nyquist bin
            v = x[h];
            v.x *= (T)0.5;
            v.y *= (T)0.5;
        }
    }
    v.x *= scale;
    v.y *= scale;
    Y[c * num + k] = v;
}

}  // namespace

int fft_c2c(tetra_ctx *ctx, bool inverse, bool dbl, size_t len, size_t batch, size_t istride, size_t idist,
            size_t ostride, size_t odist, void *in, void *out) {
    std::call_once(g_fft_once, [] { rocfft_setup(); });
    if (!ctx->fft) {
        ctx->fft = new FftCache();
        ctx->fft_free = fft_free;
    }
    auto *cache = static_cast<FftCache *>(ctx->fft);
    const bool inplace = in == out;
    size_t hit = cache->plans.size();
    for (size_t i = 0; i < cache->plans.size(); ++i) {
        const FftPlan &f = cache->plans[i];
        if (f.inverse == inverse && f.dbl == dbl && f.len == len && f.batch == batch && f.istride == istride &&
            f.idist == idist && f.ostride == ostride && f.odist == odist && f.inplace == inplace)
            hit = i;
    }
    if (hit == cache->plans.size()) {
        if (cache->plans.size() >= FFT_MAX_PLANS) {   // evict the oldest (its last use is ordered on the stream)
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            destroy_plan(cache->plans.front());
            cache->plans.erase(cache->plans.begin());
        }
        FftPlan f{inverse, dbl, len, batch, istride, idist, ostride, odist, inplace, nullptr, nullptr, 0};
        rocfft_plan_description desc = nullptr;
        if (rocfft_plan_description_create(&desc) != rocfft_status_success)
            return tetra_fail(ctx, TETRA_E_HIP, "rocfft_plan_description_create failed");
        const size_t is[1] = {istride}, os[1] = {ostride};
        rocfft_status s = rocfft_plan_description_set_data_layout(
            desc, rocfft_array_type_complex_interleaved, rocfft_array_type_complex_interleaved, nullptr, nullptr, 1, is,
            idist, 1, os, odist);
        const size_t lens[1] = {len};
        if (s == rocfft_status_success)
            s = rocfft_plan_create(&f.plan, inplace ? rocfft_placement_inplace : rocfft_placement_notinplace,
                                   inverse ? rocfft_transform_type_complex_inverse : rocfft_transform_type_complex_forward,
                                   dbl ? rocfft_precision_double : rocfft_precision_single, 1, lens, batch, desc);
        rocfft_plan_description_destroy(desc);
        if (s != rocfft_status_success) return tetra_fail(ctx, TETRA_E_HIP, "rocfft_plan_create failed (%d)", (int)s);
        rocfft_plan_get_work_buffer_size(f.plan, &f.work);
        rocfft_execution_info_create(&f.info);
        cache->plans.push_back(f);
        hit = cache->plans.size() - 1;
    }
    FftPlan &fp = cache->plans[hit];
    if (fp.work > cache->work.bytes) {
        if (cache->work.p) HIP_TRY(ctx, hipFree(cache->work.p));
        cache->work = DevBuf{};
        HIP_TRY(ctx, hipMalloc(&cache->work.p, fp.work));
        cache->work.bytes = fp.work;
    }
    if (fp.work) rocfft_execution_info_set_work_buffer(fp.info, cache->work.p, fp.work);
    rocfft_execution_info_set_stream(fp.info, ctx->stream);
    void *ib[1] = {in}, *ob[1] = {out};
    if (rocfft_execute(fp.plan, ib, inplace ? nullptr : ob, fp.info) != rocfft_status_success)
        return tetra_fail(ctx, TETRA_E_HIP, "rocfft_execute failed");
    return TETRA_OK;
}

extern "C" {

int tetra_resample(tetra_ctx *ctx, const void *x, int fmt, size_t C, size_t Nx, size_t num, void *y) {
    if (!ctx) return TETRA_E_INVALID;
    if (fmt != TETRA_CF32 && fmt != TETRA_CF64)
        return tetra_fail(ctx, TETRA_E_INVALID, "resample takes complex64 or complex128 rows");
    if (C == 0 || Nx == 0 || num == 0 || !x || !y) return tetra_fail(ctx, TETRA_E_INVALID, "empty resample request");
    const bool dbl = fmt == TETRA_CF64;
    const size_t es = dbl ? 16 : 8;
    Staging st(ctx);
    const void *xd = st.in(x, C * Nx * es);
    void *yd = st.out(y, C * num * es);
    void *X = ws(ctx, S_W1, C * Nx * es);   // spectrum of x
    if (!xd || !yd || !X) return st.finish();
    {
        PROF(ctx, "resample");
        // in place on a copy: an out-of-place rocFFT plan may use its input as scratch
        HIP_TRY(ctx, hipMemcpyAsync(X, xd, C * Nx * es, hipMemcpyDeviceToDevice, ctx->stream));
        int rc = fft_c2c(ctx, false, dbl, Nx, C, 1, Nx, 1, Nx, X, X);
        if (rc) return rc;
        const dim3 g((unsigned)((num + 255) / 256), (unsigned)C);
        if (dbl)
            hipLaunchKernelGGL((k_resample_spectrum<double2, double>), g, dim3(256), 0, ctx->stream,
                               (const double2 *)X, (long)Nx, (long)num, 1.0 / (double)Nx, (double2 *)yd);
        else
            hipLaunchKernelGGL((k_resample_spectrum<float2, float>), g, dim3(256), 0, ctx->stream, (const float2 *)X,
                               (long)Nx, (long)num, (float)(1.0 / (double)Nx), (float2 *)yd);
        HIP_TRY(ctx, hipGetLastError());
        rc = fft_c2c(ctx, true, dbl, num, C, 1, num, 1, num, yd, yd);
        if (rc) return rc;
    }
    return st.finish();
}

}  // extern "C"
