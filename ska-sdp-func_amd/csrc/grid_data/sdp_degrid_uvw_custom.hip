// MI355X-native degridding with caller-supplied uv / w kernels.
//
// Replaces src/ska-sdp-func/grid_data/sdp_degrid_uvw_custom.cpp / .cu of
// ska-sdp-func 1.2.2 (a thread per (baseline, channel, time) walking
// w_kernel_size x K x K grid cells serially). Here one wavefront owns a
// visibility: lane k takes uv tap (y, x) = (k / K, k % K) -- consecutive
// lanes read consecutive grid cells of a row, so the gather is coalesced --
// accumulates kw[z] (kv[y] (ku[x] g)) over the w taps in registers for
// every polarisation, and one wave reduction per polarisation produces the
// visibility. Coordinates and the in-grid test follow
// sdp_degrid_uvw_custom.cpp:20-62 and :134-140 operation for operation.
#include <cmath>
#include <cstdint>

#include "ska-sdp-func/grid_data/sdp_degrid_uvw_custom.h"
#include "../utility/sdp_hip.h"

namespace {

constexpr double kC0 = 299792458.0;
constexpr int kWaves = 4;
constexpr int kMaxPols = 4;

struct CParams
{
    int64_t K, KW, OS, OSW;          // uv / w kernel sizes and oversampling
    int64_t X, Y, Z, C, P;           // grid dims, channels, pols
    int64_t num_vis;                 // times x baselines x channels
    double theta, wstep, f0, df;
    int conjugate;
};

__device__ __forceinline__ double2 cmul_add(double2 acc, double k, double2 g)
{
    return make_double2(acc.x + k * g.x, acc.y + k * g.y);
}

__global__ __launch_bounds__(64 * kWaves) void k_degrid_custom(CParams p,
        const double2* __restrict__ grid, const double* __restrict__ uvw,
        const double* __restrict__ uv_kernel,
        const double* __restrict__ w_kernel, double2* __restrict__ vis)
{
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const int64_t v = blockIdx.x * (int64_t)kWaves + (threadIdx.x >> 6);
    if (v >= p.num_vis) return;
    const int64_t tb = v / p.C, c = v - tb * p.C;
    const double inv_wavelength = (p.f0 + c * p.df) / kC0;
    const double u = inv_wavelength * uvw[3 * tb];
    const double vv = inv_wavelength * uvw[3 * tb + 1];
    const double w = inv_wavelength * uvw[3 * tb + 2];
    // calculate_coordinates (.cpp:20-62).
    const int os = (int)p.OS, osw = (int)p.OSW;
    const int iox = (int)round(p.theta * u * os) + (int)(p.X / 2 + 1) * os - 1;
    const int home_x = iox / os;
    const int frac_x = os - 1 - (iox % os);
    const int ioy = (int)round(p.theta * vv * os) + (int)(p.X / 2 + 1) * os -
            1;
    const int home_y = ioy / os;
    const int frac_y = os - 1 - (ioy % os);
    const int ioz = (int)round((1.0 + w / p.wstep) * osw) + osw - 1;
    const int frac_z = osw - 1 - (ioz % osw);
    const int64_t half = p.K / 2;
    if (!(home_x > half && home_x < p.X - half && home_y > half &&
            home_y < p.Y - half))
        return;
    // A negative ioz that is not a multiple of osw gives a w-kernel row past
    // the table, which the reference reads out of bounds (undefined); such
    // visibilities are left unwritten, like those off the grid.
    if (frac_z >= osw) return;
    const double* ku = uv_kernel + (int64_t)p.K * frac_x;
    const double* kv = uv_kernel + (int64_t)p.K * frac_y;
    const double* kw = w_kernel + (int64_t)p.KW * frac_z;
    double2 acc[kMaxPols];
#pragma unroll
    for (int q = 0; q < kMaxPols; ++q) acc[q] = make_double2(0.0, 0.0);
    for (int64_t k = lane; k < p.K * p.K; k += 64)
    {
        const int64_t y = k / p.K, x = k - y * p.K;
        const int64_t gy = home_y + y - half, gx = home_x + x - half;
        const double kuv_x = ku[x], kuv_y = kv[y];
        for (int64_t z = 0; z < p.KW; ++z)
        {
            const double2* g = grid + (((c * p.Z + z) * p.Y + gy) * p.X +
                    gx) * p.P;
            const double kz = kw[z];
#pragma unroll
            for (int q = 0; q < kMaxPols; ++q)
            {
                if (q >= p.P) break;
                const double2 gv = g[q];
                const double2 t = make_double2(kuv_x * gv.x, kuv_x * gv.y);
                const double2 ty = make_double2(kuv_y * t.x, kuv_y * t.y);
                acc[q] = cmul_add(acc[q], kz, ty);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < kMaxPols; ++q)
    {
        if (q >= p.P) break;
        double re = acc[q].x, im = acc[q].y;
        for (int o = 32; o > 0; o >>= 1)
        {
            re += __shfl_xor(re, o, 64);
            im += __shfl_xor(im, o, 64);
        }
        if (lane == 0) vis[v * p.P + q] = make_double2(re, p.conjugate ? -im : im);
    }
}

} // namespace

extern "C" {

void sdp_degrid_uvw_custom(const sdp_Mem* grid, const sdp_Mem* uvw,
        const sdp_Mem* uv_kernel, const sdp_Mem* w_kernel, const double theta,
        const double wstep, const double channel_start_hz,
        const double channel_step_hz, const int32_t conjugate, sdp_Mem* vis,
        sdp_Error* status)
{
    if (*status) return;
    // sdp_data_model_get_vis_metadata + checks (.cpp:205-250).
    if (!sdp_mem_is_complex(vis))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("The visibility array must be complex");
        return;
    }
    sdp_mem_check_num_dims(vis, 4, status);
    if (*status) return;
    const int64_t T = sdp_mem_shape_dim(vis, 0), B = sdp_mem_shape_dim(vis, 1);
    const int64_t C = sdp_mem_shape_dim(vis, 2), P = sdp_mem_shape_dim(vis, 3);
    if (P != 4 && P != 1)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("The number of polarisations should be 4 or 1");
        return;
    }
    const sdp_MemLocation loc = sdp_mem_location(vis);
    sdp_mem_check_writeable(vis, status);
    if (!*status && (!sdp_mem_is_floating_point(uvw) ||
            sdp_mem_is_complex(uvw)))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("The uvw array must be real-valued");
    }
    const int64_t uvw_shape[] = {T, B, 3};
    sdp_mem_check_shape(uvw, 3, uvw_shape, status);
    sdp_mem_check_location(uvw, loc, status);
    sdp_mem_check_c_contiguity(uvw, status);
    sdp_mem_check_num_dims(uv_kernel, 2, status);
    sdp_mem_check_num_dims(w_kernel, 2, status);
    sdp_mem_check_num_dims(grid, 5, status);
    if (*status) return;
    CParams p;
    p.OS = sdp_mem_shape_dim(uv_kernel, 0);
    p.K = sdp_mem_shape_dim(uv_kernel, 1);
    p.OSW = sdp_mem_shape_dim(w_kernel, 0);
    p.KW = sdp_mem_shape_dim(w_kernel, 1);
    p.Z = sdp_mem_shape_dim(grid, 1);
    p.Y = sdp_mem_shape_dim(grid, 2);
    p.X = sdp_mem_shape_dim(grid, 3);
    const int64_t grid_shape[] = {C, p.Z, p.Y, p.X, P};
    sdp_mem_check_shape(grid, 5, grid_shape, status);
    if (*status) return;
    if (sdp_mem_location(grid) != loc || sdp_mem_location(uv_kernel) != loc ||
            sdp_mem_location(w_kernel) != loc)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Memory location mismatch");
        return;
    }
    if (sdp_mem_type(vis) != SDP_MEM_COMPLEX_DOUBLE ||
            sdp_mem_type(grid) != SDP_MEM_COMPLEX_DOUBLE ||
            sdp_mem_type(uvw) != SDP_MEM_DOUBLE ||
            sdp_mem_type(uv_kernel) != SDP_MEM_DOUBLE ||
            sdp_mem_type(w_kernel) != SDP_MEM_DOUBLE)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Currently, only double-precision data can be used");
        return;
    }
    // The flat indexing of this implementation needs C-contiguous arrays and
    // a w axis that covers the w kernel.
    sdp_mem_check_c_contiguity(grid, status);
    sdp_mem_check_c_contiguity(uv_kernel, status);
    sdp_mem_check_c_contiguity(w_kernel, status);
    sdp_mem_check_c_contiguity(vis, status);
    if (*status) return;
    if (p.Z < p.KW || p.OS < 1 || p.OSW < 1)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Grid w axis shorter than the w kernel, or empty "
                "kernel tables");
        return;
    }
    p.C = C;
    p.P = P;
    p.num_vis = T * B * C;
    p.theta = theta;
    p.wstep = wstep;
    p.f0 = channel_start_hz;
    p.df = channel_step_hz;
    p.conjugate = conjugate ? 1 : 0;
    if (p.num_vis == 0) return;
    if (!sdp_hip::device_available())
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("No GPU available for sdp_degrid_uvw_custom.");
        return;
    }
    const sdp_Mem* in[4] = {grid, uvw, uv_kernel, w_kernel};
    const void* d_in[4];
    void* tmp[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    void* d_vis = sdp_mem_data(vis);
    const size_t vis_bytes = (size_t)p.num_vis * P * 16;
    for (int k = 0; k < 4; ++k) d_in[k] = sdp_mem_data_const(in[k]);
    if (loc == SDP_MEM_CPU)
    {
        // Host arrays are staged through device memory.
        for (int k = 0; k < 5 && !*status; ++k)
        {
            const size_t bytes = k < 4 ? (size_t)sdp_mem_num_elements(in[k]) *
                    sdp_mem_type_size(sdp_mem_type(in[k])) : vis_bytes;
            if (hipMalloc(&tmp[k], bytes ? bytes : 1) != hipSuccess)
            {
                *status = SDP_ERR_MEM_ALLOC_FAILURE;
                SDP_LOG_ERROR("Cannot stage %zu bytes in device memory",
                        bytes);
                break;
            }
            SDP_HIP_CHECK(hipMemcpy(tmp[k], k < 4 ? d_in[k] : d_vis, bytes,
                    hipMemcpyHostToDevice), status);
            if (k < 4) d_in[k] = tmp[k];
        }
    }
    double2* out = (double2*)(loc == SDP_MEM_CPU ? tmp[4] : d_vis);
    if (!*status)
    {
        const unsigned blocks = (unsigned)((p.num_vis + kWaves - 1) / kWaves);
        k_degrid_custom<<<blocks, 64 * kWaves>>>(p, (const double2*)d_in[0],
                (const double*)d_in[1], (const double*)d_in[2],
                (const double*)d_in[3], out);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    if (loc == SDP_MEM_CPU)
    {
        if (!*status)
            SDP_HIP_CHECK(hipMemcpy(d_vis, tmp[4], vis_bytes,
                    hipMemcpyDeviceToHost), status);
        for (void* t : tmp) (void)hipFree(t);
    }
}

} // extern "C"
