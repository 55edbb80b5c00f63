// MI355X-native point-source DFT prediction (sdp_dft_point_v00 / v01).
//
// Replaces src/ska-sdp-func/visibility/sdp_dft.cpp / .cu of ska-sdp-func
// 1.2.2. The work is (visibilities x components) phasors, compute-bound on
// the double-precision sincos. A workgroup of 256 threads covers 256
// baselines of one (time, channel): the channel's inverse wavelength and
// flux column are shared, so components are staged through LDS in chunks
// of 256 (directions and the chunk's fluxes for this channel, one
// coalesced load each) and every thread accumulates its visibility's
// polarisations in registers over the chunk. The phase and phasor follow
// sdp_dft.cpp:49-77 (v00) and :291-318 (v01) operation for operation.
// v01 by default takes k_dft_rec (below): one thread per (time, baseline)
// and 8 channels, the phasor advanced across channels by a complex
// multiplication instead of a sincos per channel, and the flux products
// accumulated with fused multiply-adds (as the reference's CUDA build
// contracts them); within 1e-12 (c128) of the CPU path.
#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "ska-sdp-func/visibility/sdp_dft.h"
#include "../utility/sdp_hip.h"

namespace {

constexpr double kC0 = 299792458.0;
constexpr int kThreads = 256;

struct DftArgs
{
    int64_t S, T, B, C, P;
    double f0, df;
    const double* dir;       // [S][3]
    const double2* flux;     // [S][C][P]
    const double* uvw;       // v00: [T][B][C][3], v01: [T][B][3]
};

template<typename V> struct Cx2;
template<> struct Cx2<double> { using type = double2; };
template<> struct Cx2<float> { using type = float2; };

template<typename V, bool V01>
__global__ __launch_bounds__(kThreads) void k_dft(DftArgs a,
        typename Cx2<V>::type* __restrict__ vis)
{
#pragma clang fp contract(off)
    using C2 = typename Cx2<V>::type;
    __shared__ double s_dir[kThreads][3];
    __shared__ double2 s_flux[kThreads][4];
    const int64_t b = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    const int64_t c = blockIdx.y, t = blockIdx.z;
    const bool live = b < a.B;
    double uu = 0.0, vv = 0.0, ww = 0.0;
    if (live)
    {
        const double* p = V01 ? a.uvw + (t * a.B + b) * 3 :
                a.uvw + ((t * a.B + b) * a.C + c) * 3;
        uu = p[0];
        vv = p[1];
        ww = p[2];
    }
    const double inv_wavelength = (a.f0 + c * a.df) / kC0;
    V acc_re[4] = {0, 0, 0, 0}, acc_im[4] = {0, 0, 0, 0};
    for (int64_t s0 = 0; s0 < a.S; s0 += kThreads)
    {
        const int n = (int)min((int64_t)kThreads, a.S - s0);
        __syncthreads();
        if ((int)threadIdx.x < n)
        {
            const int64_t s = s0 + threadIdx.x;
            s_dir[threadIdx.x][0] = a.dir[3 * s];
            s_dir[threadIdx.x][1] = a.dir[3 * s + 1];
            s_dir[threadIdx.x][2] = a.dir[3 * s + 2];
            for (int q = 0; q < a.P; ++q)
                s_flux[threadIdx.x][q] = a.flux[(s * a.C + c) * a.P + q];
        }
        __syncthreads();
        if (!live) continue;
        for (int k = 0; k < n; ++k)
        {
            const double l = s_dir[k][0], m = s_dir[k][1], nn = s_dir[k][2];
            const double phase = V01 ?
                    -2.0 * M_PI * inv_wavelength * (l * uu + m * vv + nn * ww) :
                    -2.0 * M_PI * (l * uu + m * vv + nn * ww);
            double sn, cs;
            sincos(phase, &sn, &cs);
            const V pr = (V)cs, pi = (V)sn;
            for (int q = 0; q < 4; ++q)
            {
                if (q >= a.P) break;
                const V fr = (V)s_flux[k][q].x, fi = (V)s_flux[k][q].y;
                acc_re[q] += pr * fr - pi * fi;
                acc_im[q] += pr * fi + pi * fr;
            }
        }
    }
    if (!live) return;
    C2* out = vis + ((t * a.B + b) * a.C + c) * a.P;
    for (int q = 0; q < a.P; ++q)
    {
        C2 z;
        z.x = acc_re[q];
        z.y = acc_im[q];
        out[q] = z;
    }
}

// v01 with a channel recurrence. The phase is linear in the channel index
// (inv_wavelength = (f0 + c df) / c0), so a thread owns one (time,
// baseline) and kCb consecutive channels: per component it evaluates the
// phasor of the first channel exactly as the reference (one sincos of the
// reference's phase) and one sincos of the per-channel step, then advances
// the phasor by complex multiplication in double (kCb - 1 steps, a few ulp
// from the reference's per-channel sincos). Components and their fluxes
// for the thread's channels are staged through LDS, 64 at a time.
constexpr int kCb = 8;
constexpr int kSrcChunk = 64;

template<typename V>
__global__ __launch_bounds__(kThreads) void k_dft_rec(DftArgs a,
        typename Cx2<V>::type* __restrict__ vis)
{
#pragma clang fp contract(off)
    using C2 = typename Cx2<V>::type;
    __shared__ double s_dir[kSrcChunk][3];
    __shared__ double2 s_flux[kSrcChunk][kCb][4];
    const int64_t b = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.y * kCb, t = blockIdx.z;
    const int nc = (int)min((int64_t)kCb, a.C - c0);
    const bool live = b < a.B;
    double uu = 0.0, vv = 0.0, ww = 0.0;
    if (live)
    {
        const double* p = a.uvw + (t * a.B + b) * 3;
        uu = p[0];
        vv = p[1];
        ww = p[2];
    }
    const double inv_wl0 = (a.f0 + c0 * a.df) / kC0;
    const double dinv_wl = a.df / kC0;
    V acc_re[kCb][4], acc_im[kCb][4];
#pragma unroll
    for (int j = 0; j < kCb; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc_re[j][q] = acc_im[j][q] = (V)0;
    const int per_src = nc * (int)a.P;
    for (int64_t s0 = 0; s0 < a.S; s0 += kSrcChunk)
    {
        const int n = (int)min((int64_t)kSrcChunk, a.S - s0);
        __syncthreads();
        for (int k = threadIdx.x; k < n * 3; k += kThreads)
            s_dir[k / 3][k % 3] = a.dir[3 * s0 + k];
        for (int k = threadIdx.x; k < n * per_src; k += kThreads)
        {
            const int src = k / per_src, r = k - src * per_src;
            const int j = r / (int)a.P, q = r - j * (int)a.P;
            s_flux[src][j][q] = a.flux[((s0 + src) * a.C + c0 + j) * a.P + q];
        }
        __syncthreads();
        if (!live) continue;
        for (int k = 0; k < n; ++k)
        {
            const double l = s_dir[k][0], m = s_dir[k][1], nn = s_dir[k][2];
            const double dot = l * uu + m * vv + nn * ww;
            double sn, cs, dsn, dcs;
            sincos(-2.0 * M_PI * inv_wl0 * dot, &sn, &cs);
            sincos(-2.0 * M_PI * dinv_wl * dot, &dsn, &dcs);
#pragma unroll
            for (int j = 0; j < kCb; ++j)
            {
                if (j >= nc) break;
                const V pr = (V)cs, pi = (V)sn;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                {
                    if (q >= a.P) break;
                    const V fr = (V)s_flux[k][j][q].x;
                    const V fi = (V)s_flux[k][j][q].y;
                    acc_re[j][q] = fma(-pi, fi, fma(pr, fr, acc_re[j][q]));
                    acc_im[j][q] = fma(pi, fr, fma(pr, fi, acc_im[j][q]));
                }
                const double ncs = cs * dcs - sn * dsn;
                sn = cs * dsn + sn * dcs;
                cs = ncs;
            }
        }
    }
    if (!live) return;
#pragma unroll
    for (int j = 0; j < kCb; ++j)
    {
        if (j >= nc) break;
        C2* out = vis + ((t * a.B + b) * a.C + c0 + j) * a.P;
#pragma unroll
        for (int q = 0; q < 4; ++q)
        {
            if (q >= a.P) break;
            C2 z;
            z.x = acc_re[j][q];
            z.y = acc_im[j][q];
            out[q] = z;
        }
    }
}

// Checks shared by v00 / v01 (sdp_dft.cpp:108-150, :343-390).
bool check(const sdp_Mem* dir, const sdp_Mem* flux, const sdp_Mem* uvw,
        bool v01, sdp_Mem* vis, int64_t* dims, sdp_Error* status)
{
    if (*status) return false;
    if (!sdp_mem_is_complex(vis))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("The visibility array must be complex");
        return false;
    }
    sdp_mem_check_num_dims(vis, 4, status);
    if (*status) return false;
    for (int d = 0; d < 4; ++d) dims[d] = sdp_mem_shape_dim(vis, d);
    if (dims[3] != 4 && dims[3] != 1)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("The number of polarisations should be 4 or 1");
        return false;
    }
    const sdp_MemLocation loc = sdp_mem_location(vis);
    sdp_mem_check_writeable(vis, status);
    sdp_mem_check_c_contiguity(vis, status);
    sdp_mem_check_c_contiguity(dir, status);
    sdp_mem_check_c_contiguity(flux, status);
    sdp_mem_check_c_contiguity(uvw, status);
    if (*status) return false;
    if (sdp_mem_location(flux) != loc || sdp_mem_location(dir) != loc ||
            sdp_mem_location(uvw) != loc)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Memory location mismatch");
        return false;
    }
    if (!sdp_mem_is_complex(flux))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Source flux values must be complex");
        return false;
    }
    sdp_mem_check_num_dims(dir, 2, status);
    if (*status) return false;
    dims[4] = sdp_mem_shape_dim(dir, 0);
    const int64_t shape_dir[] = {dims[4], 3};
    const int64_t shape_flux[] = {dims[4], dims[2], dims[3]};
    sdp_mem_check_shape(dir, 2, shape_dir, status);
    sdp_mem_check_shape(flux, 3, shape_flux, status);
    if (v01)
    {
        const int64_t shape_uvw[] = {dims[0], dims[1], 3};
        sdp_mem_check_shape(uvw, 3, shape_uvw, status);
    }
    else
    {
        const int64_t shape_uvw[] = {dims[0], dims[1], dims[2], 3};
        sdp_mem_check_shape(uvw, 4, shape_uvw, status);
    }
    if (*status) return false;
    const sdp_MemType vt = sdp_mem_type(vis);
    if (sdp_mem_type(dir) != SDP_MEM_DOUBLE ||
            sdp_mem_type(flux) != SDP_MEM_COMPLEX_DOUBLE ||
            sdp_mem_type(uvw) != SDP_MEM_DOUBLE ||
            (vt != SDP_MEM_COMPLEX_DOUBLE && vt != SDP_MEM_COMPLEX_FLOAT))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data type(s)");
        return false;
    }
    if (!sdp_hip::device_available())
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("No GPU available for the DFT.");
        return false;
    }
    return true;
}

void dft(const sdp_Mem* dir, const sdp_Mem* flux, const sdp_Mem* uvw,
        bool v01, double f0, double df, sdp_Mem* vis, sdp_Error* status)
{
    int64_t dims[5] = {0, 0, 0, 0, 0};
    if (!check(dir, flux, uvw, v01, vis, dims, status)) return;
    DftArgs a;
    a.T = dims[0];
    a.B = dims[1];
    a.C = dims[2];
    a.P = dims[3];
    a.S = dims[4];
    a.f0 = f0;
    a.df = df;
    const bool host = sdp_mem_location(vis) == SDP_MEM_CPU;
    const sdp_Mem* in[3] = {dir, flux, uvw};
    const void* d_in[3];
    void* tmp[4] = {nullptr, nullptr, nullptr, nullptr};
    const size_t vis_bytes = (size_t)sdp_mem_num_elements(vis) *
            sdp_mem_type_size(sdp_mem_type(vis));
    void* d_vis = sdp_mem_data(vis);
    for (int k = 0; k < 3; ++k) d_in[k] = sdp_mem_data_const(in[k]);
    if (host)
    {
        for (int k = 0; k < 3 && !*status; ++k)
        {
            const size_t bytes = (size_t)sdp_mem_num_elements(in[k]) *
                    sdp_mem_type_size(sdp_mem_type(in[k]));
            if (hipMalloc(&tmp[k], bytes ? bytes : 1) != hipSuccess)
            {
                *status = SDP_ERR_MEM_ALLOC_FAILURE;
                break;
            }
            SDP_HIP_CHECK(hipMemcpy(tmp[k], d_in[k], bytes,
                    hipMemcpyHostToDevice), status);
            d_in[k] = tmp[k];
        }
        if (!*status && hipMalloc(&tmp[3], vis_bytes ? vis_bytes : 1) !=
                hipSuccess)
            *status = SDP_ERR_MEM_ALLOC_FAILURE;
    }
    void* out = host ? tmp[3] : d_vis;
    a.dir = (const double*)d_in[0];
    a.flux = (const double2*)d_in[1];
    a.uvw = (const double*)d_in[2];
    if (!*status && a.T * a.B * a.C > 0)
    {
        const dim3 grid((unsigned)((a.B + kThreads - 1) / kThreads),
                (unsigned)a.C, (unsigned)a.T);
        const dim3 grid_rec(grid.x, (unsigned)((a.C + kCb - 1) / kCb),
                (unsigned)a.T);
        const bool dbl = sdp_mem_type(vis) == SDP_MEM_COMPLEX_DOUBLE;
        // v01: the phasor recurrence over channels (one sincos per
        // channel measured 3.8 -> 6.5 ms, c128); v00 has one channel
        // frequency per (time, channel) block and keeps a sincos per phasor.
        if (v01 && dbl)
            k_dft_rec<double><<<grid_rec, kThreads>>>(a, (double2*)out);
        else if (v01)
            k_dft_rec<float><<<grid_rec, kThreads>>>(a, (float2*)out);
        else if (dbl)
            k_dft<double, false><<<grid, kThreads>>>(a, (double2*)out);
        else
            k_dft<float, false><<<grid, kThreads>>>(a, (float2*)out);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    if (host)
    {
        if (!*status)
            SDP_HIP_CHECK(hipMemcpy(d_vis, tmp[3], vis_bytes,
                    hipMemcpyDeviceToHost), status);
        for (void* p : tmp) (void)hipFree(p);
    }
}

} // namespace

extern "C" {

void sdp_dft_point_v00(const sdp_Mem* source_directions,
        const sdp_Mem* source_fluxes, const sdp_Mem* uvw_lambda,
        sdp_Mem* vis, sdp_Error* status)
{
    dft(source_directions, source_fluxes, uvw_lambda, false, 0.0, 0.0, vis,
            status);
}

void sdp_dft_point_v01(const sdp_Mem* source_directions,
        const sdp_Mem* source_fluxes, const sdp_Mem* uvw,
        const double channel_start_hz, const double channel_step_hz,
        sdp_Mem* vis, sdp_Error* status)
{
    dft(source_directions, source_fluxes, uvw, true, channel_start_hz,
            channel_step_hz, vis, status);
}

} // extern "C"
