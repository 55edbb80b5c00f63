// MI355X-native multi-scale CLEAN, Cornwell's algorithm
// (sdp_ms_clean_cornwell).
//
// Replaces src/ska-sdp-func/clean/sdp_ms_clean_cornwell.cpp of ska-sdp-func
// 1.2.2, which exists only as a CPU path (a GPU call does nothing there).
// Set-up, all on the device:
//   * scale kernels (Gaussians of sigma 3/16 scale, a delta for scale 0)
//     and the CLEAN beam, psf-sized as in the reference, are generated and
//     Fourier transformed once (rocFFT, P x P with P the power of two
//     >= 2 x psf size - 1);
//   * every convolution is the reference's sdp_fft_convolution: linear,
//     "same"-aligned to the first operand (out[i] = sum in1[k]
//     in2[i - k + (n2 - 1) / 2]), evaluated as pad -> FFT -> product ->
//     inverse FFT -> crop with the 1 / P^2 scaling, in the image type;
//   * scaled PSFs psf (*) k_s (*) k_p for every scale pair, scaled residuals
//     residual (*) k_s, and the coupling matrix diagonal (max of each
//     psf (*) k_s (*) k_s, floored at 0).
// The minor cycle is the Hogbom structure over S scales: k_ms_cycle applies
// the previous pick (component += g m kernel_m window, every scaled residual
// -= g m scaled-psf[s][m] window) and takes per-scale argmaxes of what it
// wrote; k_ms_reduce (one workgroup) reduces them, biases each scale's peak
// by its coupling, picks the scale, tests the threshold on that scale's
// residual and publishes the next pick. 64 cycles per captured graph, stop
// flag polled per graph. The arithmetic of a cycle is the reference's in
// the image type (sdp_ms_clean_cornwell.cpp:557-702: strict ">" scans from
// 0, first index on ties, gain x peak rounded to T then times the tables).
// Only real parts are kept: the reference's complex buffers are multiplied
// by real scalars only, so their imaginary parts never reach the outputs.
#include <cmath>
#include <cstdint>
#include <type_traits>
#include <vector>

#include "ska-sdp-func/clean/sdp_ms_clean_cornwell.h"
#include "../fft/fft2d.h"
#include "../utility/sdp_hip.h"
#include "clean_common.h"

namespace {

using sdp_clean::kThreads;
using sdp_clean::Peak;
using sdp_clean::better;
using sdp_clean::block_best;

constexpr int kPix = 4;
constexpr int kSpan = kThreads * kPix;
constexpr int kMaxScales = 16;
constexpr int kSyncEvery = 64;

template<typename T>
using C2 = typename std::conditional<sizeof(T) == 8, double2, float2>::type;

inline unsigned int blocks(size_t n)
{
    return (unsigned int)((n + kThreads - 1) / kThreads);
}

// Scale kernel s on an L x L table (sdp_ms_clean_cornwell.cpp:111-166).
template<typename T>
__global__ void k_scale_kern(T* k, int L, int scale)
{
    const size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x;
    if (i >= (size_t)L * L) return;
    const int x = (int)(i / L), y = (int)(i % L), c = L / 2;
    if (scale == 0)
    {
        k[i] = (x == c && y == c) ? (T)1 : (T)0;
        return;
    }
    const T sigma = (T)((3.0 / 16.0) * scale);
    const T tss = (T)(2.0 * (double)sigma * (double)sigma);
    const double d = (double)((x - c) * (x - c) + (y - c) * (y - c));
    k[i] = (T)(exp(-d / (double)tss) / (M_PI * (double)tss));
}

template<typename T>
__global__ void k_beam(T* b, int L, double sx, double sy, double th)
{
    const size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x;
    if (i >= (size_t)L * L) return;
    b[i] = (T)sdp_clean::cbeam_value((int)(i / L), (int)(i % L), L, sx, sy,
            th);
}

// n x n real -> top-left corner of a zeroed P x P complex array.
template<typename T>
__global__ void k_pad(const T* __restrict__ in, int n, C2<T>* __restrict__ buf,
        int P)
{
    const size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x;
    if (i >= (size_t)P * P) return;
    const int x = (int)(i / P), y = (int)(i % P);
    C2<T> z;
    z.x = (x < n && y < n) ? in[(size_t)x * n + y] : (T)0;
    z.y = (T)0;
    buf[i] = z;
}

template<typename T>
__global__ void k_mul(const C2<T>* __restrict__ a, const C2<T>* __restrict__ b,
        C2<T>* __restrict__ out, size_t n)
{
#pragma clang fp contract(off)
    const size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x;
    if (i >= n) return;
    const C2<T> p = a[i], q = b[i];
    C2<T> z;
    z.x = p.x * q.x - p.y * q.y;
    z.y = p.x * q.y + p.y * q.x;
    out[i] = z;
}

// out[i][j] = Re buf[i + h][j + h] / P^2 (+ add[i][j]), n x n.
template<typename T>
__global__ void k_crop(const C2<T>* __restrict__ buf, int P, int n, int h,
        T* __restrict__ out, const T* __restrict__ add)
{
    const size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x;
    if (i >= (size_t)n * n) return;
    const int x = (int)(i / n), y = (int)(i % n);
    T v = buf[(size_t)(x + h) * P + (y + h)].x / (T)((double)P * P);
    if (add) v = v + add[i];
    out[i] = v;
}

// Per-block maximum of a table (coupling matrix), floored at 0 on the host.
template<typename T>
__global__ void k_block_max(const T* __restrict__ a, size_t n,
        double* __restrict__ part)
{
    double v = 0.0;
    long long idx = 0;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n;
            i += (size_t)gridDim.x * kThreads)
        if ((double)a[i] > v) v = (double)a[i];
    block_best(v, idx);
    if (threadIdx.x == 0) part[blockIdx.x] = v;
}

struct MsState
{
    double gm;         // T(gain x biased peak) of the pending pick
    long long idx;     // its flat index
    int scale;         // its scale
    int has_pick;
    int done;
    int cycles;
};

template<typename T>
struct MsArgs
{
    T* sres;               // [S][n][n]
    const T* spsf;         // [S][S][L][L]
    const T* kern;         // [S][L][L]
    T* comp;               // [n][n]
    const T* coupling;     // [S] diagonal
    int S;
    unsigned int n, L, npix;
    T gain, thresh;
    MsState* st;
    Peak* part;            // [S][nblk]
};

template<typename T>
__global__ __launch_bounds__(kThreads) void k_ms_cycle(MsArgs<T> a)
{
#pragma clang fp contract(off)
    if (a.st->done) return;
    const bool pick = a.st->has_pick != 0;
    const T gm = (T)a.st->gm;
    const int m = a.st->scale;
    const long long pidx = a.st->idx;
    const unsigned int x0 = a.n - (unsigned int)(pidx / a.n);
    const unsigned int y0 = a.n - (unsigned int)(pidx % a.n);
    const unsigned int base = blockIdx.x * kSpan + threadIdx.x;
    const size_t LL = (size_t)a.L * a.L;
    if (pick)
    {
        const T* km = a.kern + m * LL;
        for (int k = 0; k < kPix; ++k)
        {
            const unsigned int i = base + k * kThreads;
            if (i >= a.npix) break;
            const unsigned int x = i / a.n, y = i - x * a.n;
            a.comp[i] = a.comp[i] +
                    gm * km[(size_t)(x + x0) * a.L + (y + y0)];
        }
    }
    for (int s = 0; s < a.S; ++s)
    {
        T* r = a.sres + (size_t)s * a.npix;
        const T* ps = a.spsf + ((size_t)s * a.S + m) * LL;
        double bv = -INFINITY;
        long long bi = LLONG_MAX;
        for (int k = 0; k < kPix; ++k)
        {
            const unsigned int i = base + k * kThreads;
            if (i >= a.npix) break;
            T v = r[i];
            if (pick)
            {
                const unsigned int x = i / a.n, y = i - x * a.n;
                v = v - gm * ps[(size_t)(x + x0) * a.L + (y + y0)];
                r[i] = v;
            }
            if ((double)v > bv)
            {
                bv = (double)v;
                bi = i;
            }
        }
        block_best(bv, bi);
        if (threadIdx.x == 0) a.part[(size_t)s * gridDim.x + blockIdx.x] =
                Peak{bv, bi};
    }
}

template<typename T>
__global__ __launch_bounds__(kThreads) void k_ms_reduce(MsArgs<T> a,
        unsigned int nblk)
{
#pragma clang fp contract(off)
    __shared__ double s_peak[kMaxScales];
    __shared__ long long s_idx[kMaxScales];
    if (a.st->done) return;
    for (int s = 0; s < a.S; ++s)
    {
        double bv = -INFINITY;
        long long bi = LLONG_MAX;
        for (unsigned int b = threadIdx.x; b < nblk; b += kThreads)
        {
            const Peak q = a.part[(size_t)s * nblk + b];
            if (better(q.v, q.i, bv, bi))
            {
                bv = q.v;
                bi = q.i;
            }
        }
        block_best(bv, bi);
        if (threadIdx.x == 0)
        {
            // Scan from 0 with ">" (.cpp:569-593): no positive value -> 0 at 0.
            s_peak[s] = bv > 0.0 ? bv : 0.0;
            s_idx[s] = bv > 0.0 ? bi : 0;
        }
    }
    if (threadIdx.x != 0) return;
    int m = 0;
    T mb = (T)0;
    for (int s = 0; s < a.S; ++s)
    {
        const T biased = (T)s_peak[s] / a.coupling[s];
        if (biased > mb)
        {
            mb = biased;
            m = s;
        }
    }
    if (a.sres[(size_t)m * a.npix + s_idx[m]] < a.thresh)
    {
        a.st->done = 1;
        return;
    }
    a.st->gm = (double)(T)(a.gain * mb);
    a.st->scale = m;
    a.st->idx = s_idx[m];
    a.st->has_pick = 1;
    a.st->cycles += 1;
}

// Linear "same" convolutions through one P x P rocFFT plan.
template<typename T>
struct Convolver
{
    int P = 0;
    sdp_fft::Plan2D* plan = nullptr;
    C2<T>* work = nullptr;
    hipStream_t s = nullptr;

    size_t elems() const { return (size_t)P * P; }

    // F = FFT(pad(in)), in n x n.
    void transform(const T* in, int n, C2<T>* F, sdp_Error* status)
    {
        if (*status) return;
        k_pad<T><<<blocks(elems()), kThreads, 0, s>>>(in, n, F, P);
        SDP_HIP_CHECK_LAUNCH(status);
        sdp_fft::exec_2d(plan, F, true, s, status);
    }

    // out (n1 x n1) = crop(IFFT(F1 F2)) (+ add), for an n2 x n2 in2.
    void finish(const C2<T>* F1, const C2<T>* F2, int n1, int n2, T* out,
            const T* add, sdp_Error* status)
    {
        if (*status) return;
        k_mul<T><<<blocks(elems()), kThreads, 0, s>>>(F1, F2, work, elems());
        SDP_HIP_CHECK_LAUNCH(status);
        sdp_fft::exec_2d(plan, work, false, s, status);
        if (*status) return;
        k_crop<T><<<blocks((size_t)n1 * n1), kThreads, 0, s>>>(work, P, n1,
                (n2 - 1) / 2, out, add);
        SDP_HIP_CHECK_LAUNCH(status);
    }
};

template<typename T>
struct DevBuf
{
    T* p = nullptr;
    bool alloc(size_t n, sdp_Error* status)
    {
        if (*status) return false;
        if (hipMalloc(&p, (n ? n : 1) * sizeof(T)) != hipSuccess)
        {
            p = nullptr;
            *status = SDP_ERR_MEM_ALLOC_FAILURE;
            SDP_LOG_ERROR("Unable to allocate multi-scale CLEAN buffers");
            return false;
        }
        return true;
    }
    ~DevBuf() { if (p) (void)hipFree(p); }
};

template<typename T>
void ms_clean(const T* dirty, const T* psf, const std::vector<int>& scales,
        const double beam[4], double gain, double thresh, int cycle_limit,
        int64_t n64, T* model, T* residual, T* sky, sdp_Error* status)
{
    const int n = (int)n64, L = 2 * n, S = (int)scales.size();
    int P = 1;
    while (P < 2 * L - 1) P <<= 1;
    const size_t nn = (size_t)n * n, LL = (size_t)L * L, PP = (size_t)P * P;
    hipStream_t s = nullptr;
    SDP_HIP_CHECK(hipStreamCreate(&s), status);
    Convolver<T> cv;
    cv.P = P;
    cv.s = s;
    DevBuf<C2<T> > work, fk, fb, fa, fi;
    DevBuf<T> kern, spsf, sres, tmp, coup;
    DevBuf<double> part_max;
    DevBuf<MsState> st;
    DevBuf<Peak> part;
    const unsigned int nblk = (unsigned int)((nn + kSpan - 1) / kSpan);
    work.alloc(PP, status);
    fk.alloc((size_t)S * PP, status);
    fb.alloc(PP, status);
    fa.alloc(PP, status);
    fi.alloc(PP, status);
    kern.alloc((size_t)S * LL, status);
    spsf.alloc((size_t)S * S * LL, status);
    sres.alloc((size_t)S * nn, status);
    tmp.alloc(LL, status);
    coup.alloc(S, status);
    part_max.alloc(256, status);
    st.alloc(1, status);
    part.alloc((size_t)S * nblk, status);
    if (!*status) cv.plan = sdp_fft::create_2d(P, P, sizeof(T) == 8, status);
    cv.work = work.p;
    // Scale kernels and their transforms; the CLEAN beam (psf-sized,
    // .cpp:401) and its transform.
    for (int k = 0; k < S && !*status; ++k)
    {
        k_scale_kern<T><<<blocks(LL), kThreads, 0, s>>>(kern.p + k * LL, L,
                scales[k]);
        SDP_HIP_CHECK_LAUNCH(status);
        cv.transform(kern.p + k * LL, L, fk.p + k * PP, status);
    }
    if (!*status)
    {
        k_beam<T><<<blocks(LL), kThreads, 0, s>>>(tmp.p, L, beam[0], beam[1],
                beam[2]);
        SDP_HIP_CHECK_LAUNCH(status);
        cv.transform(tmp.p, L, fb.p, status);
    }
    // Scaled PSFs (.cpp:414-486): (psf (*) k_s) (*) k_p.
    cv.transform(psf, L, fa.p, status);
    for (int a = 0; a < S && !*status; ++a)
    {
        cv.finish(fa.p, fk.p + a * PP, L, L, tmp.p, nullptr, status);
        cv.transform(tmp.p, L, fi.p, status);
        for (int b = 0; b < S && !*status; ++b)
            cv.finish(fi.p, fk.p + b * PP, L, L,
                    spsf.p + ((size_t)a * S + b) * LL, nullptr, status);
    }
    // Scaled residuals (.cpp:488-515): residual (*) k_s, n x n.
    cv.transform(dirty, n, fa.p, status);
    for (int a = 0; a < S && !*status; ++a)
        cv.finish(fa.p, fk.p + a * PP, n, L, sres.p + a * nn, nullptr, status);
    // Coupling matrix diagonal (.cpp:518-550): max(0, max psf_ss).
    std::vector<T> coupling(S);
    for (int a = 0; a < S && !*status; ++a)
    {
        k_block_max<T><<<256, kThreads, 0, s>>>(
                spsf.p + ((size_t)a * S + a) * LL, LL, part_max.p);
        SDP_HIP_CHECK_LAUNCH(status);
        double pm[256];
        SDP_HIP_CHECK(hipMemcpyAsync(pm, part_max.p, sizeof(pm),
                hipMemcpyDeviceToHost, s), status);
        SDP_HIP_CHECK(hipStreamSynchronize(s), status);
        double mx = 0.0;
        for (double v : pm) mx = v > mx ? v : mx;
        coupling[a] = (T)mx;
    }
    if (!*status)
    {
        SDP_HIP_CHECK(hipMemcpyAsync(coup.p, coupling.data(), S * sizeof(T),
                hipMemcpyHostToDevice, s), status);
        SDP_HIP_CHECK(hipMemsetAsync(st.p, 0, sizeof(MsState), s), status);
        SDP_HIP_CHECK(hipMemsetAsync(model, 0, nn * sizeof(T), s), status);
    }
    MsArgs<T> args;
    args.sres = sres.p;
    args.spsf = spsf.p;
    args.kern = kern.p;
    args.comp = model;
    args.coupling = coup.p;
    args.S = S;
    args.n = (unsigned int)n;
    args.L = (unsigned int)L;
    args.npix = (unsigned int)nn;
    args.gain = (T)gain;
    args.thresh = (T)thresh;
    args.st = st.p;
    args.part = part.p;
    auto launch_pair = [&]() {
        k_ms_cycle<T><<<nblk, kThreads, 0, s>>>(args);
        k_ms_reduce<T><<<1, kThreads, 0, s>>>(args, nblk);
    };
    if (!*status)
    {
        launch_pair();                 // first pick
        SDP_HIP_CHECK_LAUNCH(status);
    }
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    if (!*status && cycle_limit >= 2 * kSyncEvery)
    {
        SDP_HIP_CHECK(hipStreamBeginCapture(s,
                hipStreamCaptureModeThreadLocal), status);
        for (int c = 0; c < kSyncEvery && !*status; ++c) launch_pair();
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
        SDP_HIP_CHECK(hipMemcpyAsync(done_host, &st.p->done, sizeof(int),
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
            for (int k = 0; k < m; ++k) launch_pair();
            SDP_HIP_CHECK_LAUNCH(status);
            c += m;
        }
    }
    // Restore (.cpp:704-749): sky = components (*) beam + residual_0.
    cv.transform(model, n, fa.p, status);
    cv.finish(fa.p, fb.p, n, L, sky, sres.p, status);
    if (!*status)
        SDP_HIP_CHECK(hipMemcpyAsync(residual, sres.p, nn * sizeof(T),
                hipMemcpyDeviceToDevice, s), status);
    if (s) SDP_HIP_CHECK(hipStreamSynchronize(s), status);
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    if (done_host) (void)hipHostFree(done_host);
    if (cv.plan) sdp_fft::destroy_2d(cv.plan);
    if (s) (void)hipStreamDestroy(s);
}

double beam_value(const sdp_Mem* m, int k, sdp_Error* status)
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

bool check_args(const sdp_Mem* dirty, const sdp_Mem* psf,
        const sdp_Mem* beam, const sdp_Mem* scales, int cycle_limit,
        const sdp_Mem* model, const sdp_Mem* res, const sdp_Mem* sky,
        sdp_Error* status)
{
    // sdp_ms_clean_cornwell.cpp:787-871, in the same order.
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
    if (sdp_mem_type(scales) != SDP_MEM_INT)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("The scale list must be a list of 4 byte integers");
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
    // Beyond the reference, which indexes these unchecked: square images,
    // a PSF twice the image size, 1..16 scales, matching types and
    // locations, a real beam description, a positive cycle limit.
    const sdp_MemType t = sdp_mem_type(dirty);
    if (t != SDP_MEM_DOUBLE && t != SDP_MEM_FLOAT)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data type");
        return false;
    }
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
    if (sdp_mem_shape_dim(dirty, 1) != n ||
            sdp_mem_shape_dim(psf, 0) != 2 * n ||
            sdp_mem_shape_dim(psf, 1) != 2 * n)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("Images must be square and the PSF twice the size of "
                "the dirty image");
        return false;
    }
    const int64_t S = sdp_mem_num_elements(scales);
    if (S < 1 || S > kMaxScales || cycle_limit < 1 || n < 1 || n > 8192)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Need 1..16 scales, cycle_limit > 0 and an image of "
                "at most 8192^2");
        return false;
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
    if (!sdp_hip::device_available())
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("No GPU available for multi-scale CLEAN.");
        return false;
    }
    return true;
}

} // namespace

extern "C" void sdp_ms_clean_cornwell(const sdp_Mem* dirty_img,
        const sdp_Mem* psf, const sdp_Mem* cbeam_details,
        const sdp_Mem* scale_list, const double loop_gain,
        const double threshold, const int cycle_limit, sdp_Mem* clean_model,
        sdp_Mem* residual, sdp_Mem* skymodel, sdp_Error* status)
{
    if (*status) return;
    if (!check_args(dirty_img, psf, cbeam_details, scale_list, cycle_limit,
            clean_model, residual, skymodel, status))
        return;
    double beam[4];
    for (int k = 0; k < 4; ++k) beam[k] = beam_value(cbeam_details, k, status);
    std::vector<int> scales((size_t)sdp_mem_num_elements(scale_list));
    if (sdp_mem_location(scale_list) == SDP_MEM_GPU)
        SDP_HIP_CHECK(hipMemcpy(scales.data(),
                sdp_mem_data_const(scale_list), scales.size() * sizeof(int),
                hipMemcpyDeviceToHost), status);
    else
        for (size_t k = 0; k < scales.size(); ++k)
            scales[k] = ((const int*)sdp_mem_data_const(scale_list))[k];
    if (*status) return;
    const int64_t n = sdp_mem_shape_dim(dirty_img, 0);
    const bool dbl = sdp_mem_type(dirty_img) == SDP_MEM_DOUBLE;
    const size_t img = (size_t)n * n * (dbl ? 8 : 4);
    const bool host = sdp_mem_location(dirty_img) == SDP_MEM_CPU;
    // [0] dirty, [1] psf, [2] model, [3] residual, [4] skymodel
    void* d[5] = {(void*)sdp_mem_data_const(dirty_img),
            (void*)sdp_mem_data_const(psf), sdp_mem_data(clean_model),
            sdp_mem_data(residual), sdp_mem_data(skymodel)};
    void* staged[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    if (host)
    {
        const size_t bytes[5] = {img, 4 * img, img, img, img};
        for (int k = 0; k < 5 && !*status; ++k)
        {
            if (hipMalloc(&staged[k], bytes[k]) != hipSuccess)
            {
                *status = SDP_ERR_MEM_ALLOC_FAILURE;
                SDP_LOG_ERROR("Unable to allocate device images");
            }
        }
        if (!*status)
        {
            SDP_HIP_CHECK(hipMemcpy(staged[0], d[0], img,
                    hipMemcpyHostToDevice), status);
            SDP_HIP_CHECK(hipMemcpy(staged[1], d[1], 4 * img,
                    hipMemcpyHostToDevice), status);
        }
    }
    void* v[5];
    for (int k = 0; k < 5; ++k) v[k] = host ? staged[k] : d[k];
    if (!*status)
    {
        if (dbl)
            ms_clean<double>((const double*)v[0], (const double*)v[1], scales,
                    beam, loop_gain, threshold, cycle_limit, n, (double*)v[2],
                    (double*)v[3], (double*)v[4], status);
        else
            ms_clean<float>((const float*)v[0], (const float*)v[1], scales,
                    beam, loop_gain, threshold, cycle_limit, n, (float*)v[2],
                    (float*)v[3], (float*)v[4], status);
    }
    if (host)
    {
        for (int k = 2; k < 5 && !*status; ++k)
            SDP_HIP_CHECK(hipMemcpy(d[k], staged[k], img,
                    hipMemcpyDeviceToHost), status);
        for (void* p : staged) (void)hipFree(p);
    }
}
