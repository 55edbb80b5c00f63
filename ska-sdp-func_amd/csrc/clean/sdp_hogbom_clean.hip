// MI355X-native Hogbom CLEAN (sdp_hogbom_clean).
//
// Replaces src/ska-sdp-func/clean/sdp_hogbom_clean.cpp / .cu of
// ska-sdp-func 1.2.2. The CLEAN loop is inherently sequential: every cycle
// needs the maximum of the residual left by the previous one. The
// reference GPU path spends each cycle on a cascade of argmax launches,
// two memsets, a single-thread launch for the component and a PSF
// subtraction launch, with a host round trip every 100 cycles. Here one
// cycle is two launches, captured kSyncEvery cycles at a time in a graph:
//   * k_clean_cycle: every workgroup subtracts loop_gain * peak * PSF
//     (shifted to the previous peak) from its 1024 residual pixels and
//     takes the argmax of what it wrote while the values are in registers;
//   * k_clean_reduce (one workgroup) reduces the per-workgroup partials,
//     adds the previous peak's component and publishes the new peak, or
//     the stop flag when it is below threshold.
// The residual is read and written once per cycle (HBM/L2-bound, 3 x 4 or
// 3 x 8 bytes per pixel with the PSF window), and the host looks at the
// stop flag once per graph launch only; launches after the stop are
// no-ops. Arithmetic follows the reference CPU path
// (sdp_hogbom_clean.cpp:183-240): first maximum in flat order, products in
// double, one rounding to the image type per update, so the components and
// the residual are bit-identical to it.
// Restoration: the non-zero components are compacted in index order and
// k_restore convolves them with the CLEAN beam per 16 x 16 output tile
// (components whose beam window misses the tile are dropped by a wave
// ballot), which is the reference's FFT convolution (sdp_fft_convolution
// .cpp:127-244, "same" alignment: out[i] = sum in1[k] beam[i - k +
// (SIZE - 1) / 2]) evaluated directly; the skymodel is that plus the
// residual.
#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "ska-sdp-func/clean/sdp_hogbom_clean.h"
#include "../utility/sdp_hip.h"
#include "clean_common.h"

namespace {

using sdp_clean::kThreads;
using sdp_clean::kWaves;
using sdp_clean::Peak;
using sdp_clean::better;
using sdp_clean::block_best;
constexpr int kPix = 4;                    // residual pixels per thread
constexpr int kSpan = kThreads * kPix;     // pixels per workgroup
constexpr int kTile = 16;                  // restore tile edge
constexpr int kSyncEvery = 64;             // cycles between stop checks

struct CleanState
{
    double peak;       // current maximum of the residual
    long long idx;     // its flat index
    int done;          // stop flag (below threshold / nothing left)
    int cycles;        // cycles performed
};

template<typename T>
struct CleanArgs
{
    T* res;
    const T* psf;      // [2n][2n]
    T* model;
    unsigned int n;
    unsigned int npix;
    T gain, thresh;
    CleanState* st;
    Peak* part;        // [gridDim.x]
};

// SUB = false: initial peak search only.
template<typename T, bool SUB>
__global__ __launch_bounds__(kThreads) void k_clean_cycle(CleanArgs<T> a)
{
#pragma clang fp contract(off)
    if (SUB && a.st->done) return;
    double ghd = 0.0;
    long long pidx = 0;
    unsigned int x_off = 0, y_off = 0;
    if (SUB)
    {
        pidx = a.st->idx;
        ghd = (double)a.gain * a.st->peak;
        x_off = a.n - (unsigned int)(pidx / a.n);
        y_off = a.n - (unsigned int)(pidx % a.n);
    }
    double bv = -INFINITY;
    long long bi = LLONG_MAX;
    const unsigned int base = blockIdx.x * kSpan + threadIdx.x;
    // All loads of the thread's pixels first (the residual stores cannot
    // be reordered above later PSF loads by the compiler otherwise).
    T r[kPix], pv[kPix];
#pragma unroll
    for (int k = 0; k < kPix; ++k)
    {
        const unsigned int i = base + k * kThreads;
        r[k] = pv[k] = (T)0;
        if (i < a.npix)
        {
            r[k] = a.res[i];
            if (SUB)
            {
                const unsigned int x = i / a.n, y = i - x * a.n;
                pv[k] = a.psf[(size_t)(x + x_off) * (2 * a.n) + (y + y_off)];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kPix; ++k)
    {
        const unsigned int i = base + k * kThreads;
        if (i >= a.npix) break;
        if (SUB)
        {
            r[k] = (T)((double)r[k] - ghd * (double)pv[k]);
            a.res[i] = r[k];
        }
        if ((double)r[k] > bv)
        {
            bv = (double)r[k];
            bi = i;
        }
    }
    block_best(bv, bi);
    if (threadIdx.x == 0) a.part[blockIdx.x] = Peak{bv, bi};
}

// One workgroup: reduce the per-workgroup partials of the cycle that just
// ran, add the previous peak's component, publish the new peak / stop.
// A separate launch rather than a last-arriving-workgroup epilogue: the
// agent-scope release fence that epilogue needs writes back the XCD's L2
// once per workgroup, which cost more than this launch (measured 27 vs
// ~10 us per cycle at 1024^2).
template<typename T, bool SUB>
__global__ __launch_bounds__(kThreads) void k_clean_reduce(CleanArgs<T> a,
        unsigned int nblk)
{
#pragma clang fp contract(off)
    if (SUB && a.st->done) return;
    const long long pidx = a.st->idx;
    double bv = -INFINITY;
    long long bi = LLONG_MAX;
    for (unsigned int b = threadIdx.x; b < nblk; b += kThreads)
    {
        const Peak q = a.part[b];
        if (better(q.v, q.i, bv, bi))
        {
            bv = q.v;
            bi = q.i;
        }
    }
    block_best(bv, bi);
    if (threadIdx.x == 0)
    {
        if (SUB)
        {
            // sdp_hogbom_clean.cpp:212-215: the product in double, rounded
            // to T, added in T.
            a.model[pidx] = a.model[pidx] +
                    (T)((double)a.gain * a.st->peak);
            a.st->cycles += 1;
        }
        a.st->peak = bv;
        a.st->idx = bi;
        if (bi == LLONG_MAX || bv < (double)a.thresh) a.st->done = 1;
    }
}

template<typename T, bool SUB>
void launch_cycle(const CleanArgs<T>& a, unsigned int nblk, hipStream_t s)
{
    k_clean_cycle<T, SUB><<<nblk, kThreads, 0, s>>>(a);
    k_clean_reduce<T, SUB><<<1, kThreads, 0, s>>>(a, nblk);
}

// CLEAN beam table (sdp_hogbom_clean.cpp:33-80), rounded to the image type
// as the reference stores it.
template<typename T>
__global__ void k_cbeam(double* cb, int nb, double sx, double sy,
        double theta_deg)
{
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= nb * nb) return;
    cb[i] = (double)(T)sdp_clean::cbeam_value(i / nb, i % nb, nb, sx, sy,
            theta_deg);
}

template<typename T>
struct NonZero
{
    const T* m;
    __device__ __forceinline__ bool operator()(const int& i) const
    {
        return m[i] != (T)0;
    }
};

template<typename T>
__global__ __launch_bounds__(kThreads) void k_restore(const int* comp,
        const int* ncomp_ptr, const T* model, const double* cb, int nb,
        int n, const T* res, T* sky)
{
    __shared__ int s_x[kThreads], s_y[kThreads];
    __shared__ double s_v[kThreads];
    __shared__ int s_cnt[kWaves];
    const int h = (nb - 1) / 2;
    const int tx0 = blockIdx.y * kTile, ty0 = blockIdx.x * kTile;
    const int x = tx0 + threadIdx.x / kTile, y = ty0 + threadIdx.x % kTile;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ncomp = *ncomp_ptr;
    double acc = 0.0;
    for (int c0 = 0; c0 < ncomp; c0 += kThreads)
    {
        const int j = c0 + threadIdx.x;
        bool hit = false;
        int cx = 0, cy = 0;
        double v = 0.0;
        if (j < ncomp)
        {
            const int p = comp[j];
            cx = p / n;
            cy = p - cx * n;
            hit = cx - h <= tx0 + kTile - 1 && cx - h + nb - 1 >= tx0 &&
                    cy - h <= ty0 + kTile - 1 && cy - h + nb - 1 >= ty0;
            if (hit) v = (double)model[p];
        }
        const unsigned long long m = __ballot(hit);
        const int before = __popcll(m & ((1ull << lane) - 1));
        __syncthreads();              // previous chunk fully consumed
        if (lane == 0) s_cnt[w] = __popcll(m);
        __syncthreads();
        int off = 0, total = 0;
        for (int k = 0; k < kWaves; ++k)
        {
            off += (k < w) ? s_cnt[k] : 0;
            total += s_cnt[k];
        }
        if (hit)
        {
            s_x[off + before] = cx;
            s_y[off + before] = cy;
            s_v[off + before] = v;
        }
        __syncthreads();
        for (int k = 0; k < total; ++k)
        {
            const int dx = x - s_x[k] + h, dy = y - s_y[k] + h;
            if (dx >= 0 && dx < nb && dy >= 0 && dy < nb)
                acc += s_v[k] * cb[dx * nb + dy];
        }
    }
    if (x < n && y < n)
    {
        const size_t i = (size_t)x * n + y;
        const T conv = (T)acc;
        sky[i] = conv + res[i];
    }
}

double read_scalar(const sdp_Mem* m, int k, sdp_Error* status)
{
    const bool dbl = sdp_mem_type(m) == SDP_MEM_DOUBLE;
    const size_t sz = dbl ? 8 : 4;
    const char* p = (const char*)sdp_mem_data_const(m) + k * sz;
    double d = 0.0;
    float f = 0.0f;
    if (sdp_mem_location(m) == SDP_MEM_GPU)
        SDP_HIP_CHECK(hipMemcpy(dbl ? (void*)&d : (void*)&f, p, sz,
                hipMemcpyDeviceToHost), status);
    else if (dbl)
        d = *(const double*)p;
    else
        f = *(const float*)p;
    return dbl ? d : (double)f;
}

template<typename T>
void clean(T* res, const T* psf, T* model, T* sky, int64_t n, double gain,
        double thresh, int cycle_limit, const double beam[4],
        sdp_Error* status)
{
    const unsigned int npix = (unsigned int)(n * n);
    const unsigned int nblk = (npix + kSpan - 1) / kSpan;
    const int nb = (int)beam[3];
    const int max_comp = (int)((int64_t)npix < cycle_limit ? npix :
            cycle_limit);
    CleanState* st = nullptr;
    Peak* part = nullptr;
    double* cb = nullptr;
    int* comp = nullptr;
    int* ncomp = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    const hipcub::CountingInputIterator<int> idx(0);
    const NonZero<T> nz{model};
    SDP_HIP_CHECK(hipcub::DeviceSelect::If(nullptr, tmp_bytes, idx,
            (int*)nullptr, (int*)nullptr, (int)npix, nz), status);
    if (hipMalloc(&st, sizeof(CleanState)) != hipSuccess ||
            hipMalloc(&part, nblk * sizeof(Peak)) != hipSuccess ||
            hipMalloc(&cb, (size_t)nb * nb * sizeof(double)) != hipSuccess ||
            hipMalloc(&comp, (size_t)max_comp * sizeof(int)) != hipSuccess ||
            hipMalloc(&ncomp, sizeof(int)) != hipSuccess ||
            hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 1) != hipSuccess)
    {
        *status = SDP_ERR_MEM_ALLOC_FAILURE;
        SDP_LOG_ERROR("Unable to allocate CLEAN work buffers");
    }
    if (!*status)
    {
        SDP_HIP_CHECK(hipMemset(st, 0, sizeof(CleanState)), status);
        SDP_HIP_CHECK(hipMemset(model, 0, (size_t)npix * sizeof(T)), status);
    }
    CleanArgs<T> a;
    a.res = res;
    a.psf = psf;
    a.model = model;
    a.n = (unsigned int)n;
    a.npix = npix;
    a.gain = (T)gain;
    a.thresh = (T)thresh;
    a.st = st;
    a.part = part;
    // A blocking stream: ordered after the caller's null-stream work.
    hipStream_t s = nullptr;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    if (!*status) SDP_HIP_CHECK(hipStreamCreate(&s), status);
    if (!*status)
    {
        launch_cycle<T, false>(a, nblk, s);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    // kSyncEvery cycles captured once into a graph: one submission per
    // stop check instead of one per cycle.
    if (!*status && cycle_limit >= 2 * kSyncEvery)
    {
        SDP_HIP_CHECK(hipStreamBeginCapture(s,
                hipStreamCaptureModeThreadLocal), status);
        for (int c = 0; c < kSyncEvery && !*status; ++c)
            launch_cycle<T, true>(a, nblk, s);
        SDP_HIP_CHECK(hipStreamEndCapture(s, &graph), status);
        if (!*status)
            SDP_HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr,
                    nullptr, 0), status);
    }
    int* done_host = nullptr;
    if (!*status)
        SDP_HIP_CHECK(hipHostMalloc((void**)&done_host, sizeof(int),
                hipHostMallocDefault), status);
    for (int c = 0; c < cycle_limit && !*status;)
    {
        SDP_HIP_CHECK(hipMemcpyAsync(done_host, &st->done, sizeof(int),
                hipMemcpyDeviceToHost, s), status);
        SDP_HIP_CHECK(hipStreamSynchronize(s), status);
        if (*status || *done_host) break;
        if (exec && cycle_limit - c >= kSyncEvery)
        {
            SDP_HIP_CHECK(hipGraphLaunch(exec, s), status);
            c += kSyncEvery;
        }
        else
        {
            const int m = cycle_limit - c < kSyncEvery ? cycle_limit - c :
                    kSyncEvery;
            for (int k = 0; k < m; ++k)
                launch_cycle<T, true>(a, nblk, s);
            SDP_HIP_CHECK_LAUNCH(status);
            c += m;
        }
    }
    if (!*status)
    {
        k_cbeam<T><<<sdp_hip::blocks_for((long long)nb * nb, kThreads),
                kThreads, 0, s>>>(cb, nb, beam[0], beam[1], beam[2]);
        SDP_HIP_CHECK_LAUNCH(status);
        SDP_HIP_CHECK(hipcub::DeviceSelect::If(tmp, tmp_bytes, idx, comp,
                ncomp, (int)npix, nz, s), status);
        const unsigned int nt = (unsigned int)((n + kTile - 1) / kTile);
        k_restore<T><<<dim3(nt, nt), kThreads, 0, s>>>(comp, ncomp, model,
                cb, nb, (int)n, res, sky);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    if (s) SDP_HIP_CHECK(hipStreamSynchronize(s), status);
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    if (s) (void)hipStreamDestroy(s);
    if (done_host) (void)hipHostFree(done_host);
    int cycles = 0;
    if (!*status)
    {
        SDP_HIP_CHECK(hipMemcpy(&cycles, &st->cycles, sizeof(int),
                hipMemcpyDeviceToHost), status);
        SDP_LOG_DEBUG("Hogbom CLEAN: %d cycles", cycles);
    }
    (void)hipFree(st);
    (void)hipFree(part);
    (void)hipFree(cb);
    (void)hipFree(comp);
    (void)hipFree(ncomp);
    (void)hipFree(tmp);
}

bool check_args(const sdp_Mem* dirty, const sdp_Mem* psf,
        const sdp_Mem* beam, double loop_gain, int cycle_limit,
        const sdp_Mem* model, const sdp_Mem* res, const sdp_Mem* sky,
        sdp_Error* status)
{
    // sdp_hogbom_clean.cpp:746-858, in the same order.
    const int64_t n = sdp_mem_shape_dim(dirty, 0);
    if (sdp_mem_is_read_only(sky))
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("Output is not writable");
        return false;
    }
    if (sdp_mem_location(dirty) != sdp_mem_location(sky))
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Memory location mismatch");
        return false;
    }
    if (sdp_mem_type(dirty) != sdp_mem_type(psf))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("The Dirty image and PSF must be of the same data type");
        return false;
    }
    if (sdp_mem_type(dirty) != sdp_mem_type(sky))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("The input and output must be of the same data type");
        return false;
    }
    const struct { const sdp_Mem* m; const char* what; } same[] = {
        {model, "The CLEAN model and the dirty image must be the same size"},
        {res, "The residual image and the dirty image must be the same size"},
        {sky, "The skymodel image and the dirty image must be the same size"}
    };
    for (const auto& s : same)
    {
        if (sdp_mem_shape_dim(s.m, 0) != n)
        {
            *status = SDP_ERR_RUNTIME;
            SDP_LOG_ERROR("%s", s.what);
            return false;
        }
    }
    if (sdp_mem_shape_dim(beam, 0) != 4)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("The array describing the CLEAN beam must include "
                "BMAJ, BMIN, THETA and SIZE");
        return false;
    }
    if (n != sdp_mem_shape_dim(dirty, 1))
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("Dirty image array must be square shaped");
        return false;
    }
    if (sdp_mem_shape_dim(psf, 0) != sdp_mem_shape_dim(psf, 1))
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("PSF array must be square shaped");
        return false;
    }
    if (sdp_mem_shape_dim(psf, 0) != 2 * n)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("PSF array dimensions must be double the Dirty image "
                "array dimensions");
        return false;
    }
    if (cycle_limit < 1)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("Number of cycles to perform must be > 0");
        return false;
    }
    if (loop_gain <= 0)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("Loop gain must be > 0");
        return false;
    }
    const sdp_MemType t = sdp_mem_type(dirty);
    if (t != SDP_MEM_DOUBLE && t != SDP_MEM_FLOAT)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data type");
        return false;
    }
    // Beyond the reference (which indexes these unchecked): the component
    // map and residual must match the dirty image, all images 2-D,
    // C-contiguous and in one location, the beam description real.
    const sdp_Mem* imgs[] = {dirty, psf, model, res, sky};
    for (const sdp_Mem* m : imgs)
    {
        sdp_mem_check_num_dims(m, 2, status);
        sdp_mem_check_c_contiguity(m, status);
        if (*status) return false;
        if (sdp_mem_type(m) != t)
        {
            *status = SDP_ERR_DATA_TYPE;
            SDP_LOG_ERROR("All images must have the dirty image's data type");
            return false;
        }
        if (sdp_mem_location(m) != sdp_mem_location(dirty))
        {
            *status = SDP_ERR_MEM_LOCATION;
            SDP_LOG_ERROR("Memory location mismatch");
            return false;
        }
    }
    sdp_mem_check_writeable(model, status);
    sdp_mem_check_writeable(res, status);
    if (*status) return false;
    if (sdp_mem_type(beam) != SDP_MEM_DOUBLE &&
            sdp_mem_type(beam) != SDP_MEM_FLOAT)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("The CLEAN beam description must be real");
        return false;
    }
    if (n > 32768)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Images larger than 32768 x 32768 are not supported");
        return false;
    }
    if (!sdp_hip::device_available())
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("No GPU available for Hogbom CLEAN.");
        return false;
    }
    return true;
}

} // namespace

extern "C" void sdp_hogbom_clean(const sdp_Mem* dirty_img, const sdp_Mem* psf,
        const sdp_Mem* cbeam_details, const double loop_gain,
        const double threshold, const int cycle_limit, sdp_Mem* clean_model,
        sdp_Mem* residual, sdp_Mem* skymodel, sdp_Error* status)
{
    if (*status) return;
    if (!check_args(dirty_img, psf, cbeam_details, loop_gain, cycle_limit,
            clean_model, residual, skymodel, status))
        return;
    double beam[4];
    for (int k = 0; k < 4; ++k) beam[k] = read_scalar(cbeam_details, k, status);
    if (*status) return;
    if ((int64_t)beam[3] < 1 || beam[3] > 32767)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("The CLEAN beam size must be in [1, 32767]");
        return;
    }
    const int64_t n = sdp_mem_shape_dim(dirty_img, 0);
    if (n == 0) return;              // empty images: nothing to clean
    const bool dbl = sdp_mem_type(dirty_img) == SDP_MEM_DOUBLE;
    const size_t esz = dbl ? 8 : 4;
    const size_t img_bytes = (size_t)n * n * esz;
    const bool host = sdp_mem_location(dirty_img) == SDP_MEM_CPU;
    // Device views: [0] residual, [1] psf, [2] model, [3] skymodel.
    void* d[4] = {sdp_mem_data(residual), (void*)sdp_mem_data_const(psf),
            sdp_mem_data(clean_model), sdp_mem_data(skymodel)};
    void* staged[4] = {nullptr, nullptr, nullptr, nullptr};
    if (host)
    {
        const size_t bytes[4] = {img_bytes, 4 * img_bytes, img_bytes,
                img_bytes};
        for (int k = 0; k < 4 && !*status; ++k)
        {
            if (hipMalloc(&staged[k], bytes[k]) != hipSuccess)
            {
                *status = SDP_ERR_MEM_ALLOC_FAILURE;
                SDP_LOG_ERROR("Unable to allocate device images");
            }
        }
        if (!*status)
        {
            SDP_HIP_CHECK(hipMemcpy(staged[0],
                    sdp_mem_data_const(dirty_img), img_bytes,
                    hipMemcpyHostToDevice), status);
            SDP_HIP_CHECK(hipMemcpy(staged[1], sdp_mem_data_const(psf),
                    4 * img_bytes, hipMemcpyHostToDevice), status);
        }
        for (int k = 0; k < 4; ++k) d[k] = staged[k];
    }
    else
    {
        // residual = dirty image (sdp_hogbom_clean.cpp:863, :381).
        SDP_HIP_CHECK(hipMemcpy(d[0], sdp_mem_data_const(dirty_img),
                img_bytes, hipMemcpyDeviceToDevice), status);
    }
    if (!*status)
    {
        if (dbl)
            clean<double>((double*)d[0], (const double*)d[1], (double*)d[2],
                    (double*)d[3], n, loop_gain, threshold, cycle_limit, beam,
                    status);
        else
            clean<float>((float*)d[0], (const float*)d[1], (float*)d[2],
                    (float*)d[3], n, loop_gain, threshold, cycle_limit, beam,
                    status);
    }
    if (host)
    {
        if (!*status)
        {
            SDP_HIP_CHECK(hipMemcpy(sdp_mem_data(residual), staged[0],
                    img_bytes, hipMemcpyDeviceToHost), status);
            SDP_HIP_CHECK(hipMemcpy(sdp_mem_data(clean_model), staged[2],
                    img_bytes, hipMemcpyDeviceToHost), status);
            SDP_HIP_CHECK(hipMemcpy(sdp_mem_data(skymodel), staged[3],
                    img_bytes, hipMemcpyDeviceToHost), status);
        }
        for (void* p : staged) (void)hipFree(p);
    }
}
