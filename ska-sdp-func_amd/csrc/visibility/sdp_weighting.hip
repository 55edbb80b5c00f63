// MI355X-native visibility weighting (uniform, Briggs / robust).
//
// Replaces src/ska-sdp-func/visibility/sdp_weighting.cpp / .cu of
// ska-sdp-func 1.2.2. The reference walks (time, baseline, channel) three
// times in nested CPU loops (grid write :18-76, sums :80-137, read
// :158-284) or launches one thread per (baseline, channel, time) with a
// 128 x 2 x 2 block. Here every pass is one flat launch over visibilities
// (thread = (time, baseline, channel), polarisations in the thread, so the
// weight rows are read and written as contiguous runs), with the
// reference's cell arithmetic in double operation for operation:
//   1. k_grid_write: grid[cell][pol] += in (device float/double atomics);
//   2. k_grid_sums (Briggs): sum_vis grid and sum_vis grid^2 with wave +
//      workgroup reductions in double and one atomic per workgroup;
//   3. k_read_uniform / k_read_briggs: out = 1 / grid, or
//      out = in / (1 + R grid) with R formed on the device from the sums and
//      the host-computed numerator (5 10^-robust)^2 (glibc pow, as the
//      reference).
// HBM-bound gather/scatter: per visibility and polarisation one weight
// read, one grid atomic, one grid read (two for Briggs) and one weight
// write; uvw is read once per channel from L2.
#include <cmath>
#include <cstdint>

#include "ska-sdp-func/visibility/sdp_weighting.h"
#include "../utility/sdp_hip.h"

namespace {

constexpr double kC0 = 299792458.0;
constexpr int kThreads = 256;

struct WParams
{
    int64_t num_vis;     // times x baselines x channels
    int64_t C, P, G;
    double max_abs_uv;
    const double* uvw;   // [times * baselines][3]
    const double* freq;  // [C]
};

// Cell offset (into grid[u][v][pol]) of visibility v, or -1 off the grid
// (sdp_weighting.cpp:40-57).
__device__ __forceinline__ int64_t cell_of(const WParams& p, int64_t v)
{
#pragma clang fp contract(off)
    const int64_t tb = v / p.C, c = v - tb * p.C;
    const double inv_wavelength = p.freq[c] / kC0;
    const double grid_u = p.uvw[3 * tb] * inv_wavelength;
    const double grid_v = p.uvw[3 * tb + 1] * inv_wavelength;
    const int64_t half = p.G / 2;
    const int64_t iu = (int64_t)(floor(grid_u / p.max_abs_uv * (double)half) +
            (double)half);
    const int64_t iv = (int64_t)(floor(grid_v / p.max_abs_uv * (double)half) +
            (double)half);
    if (iu < 0 || iv < 0 || iu >= p.G || iv >= p.G) return -1;
    return (iu * p.G + iv) * p.P;
}

template<typename W>
__global__ __launch_bounds__(kThreads) void k_grid_write(WParams p,
        W* __restrict__ grid, const W* __restrict__ in)
{
    const int64_t v = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (v >= p.num_vis) return;
    const int64_t cell = cell_of(p, v);
    if (cell < 0) return;
    for (int64_t pol = 0; pol < p.P; ++pol)
        unsafeAtomicAdd(&grid[cell + pol], in[v * p.P + pol]);
}

__device__ __forceinline__ double wave_sum(double x)
{
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// sums[0] += sum_vis grid, sums[1] += sum_vis (W)(grid * grid)
// (sdp_weighting.cpp:127-133: the square is formed in the weight type).
template<typename W>
__global__ __launch_bounds__(kThreads) void k_grid_sums(WParams p,
        const W* __restrict__ grid, double* __restrict__ sums)
{
#pragma clang fp contract(off)
    __shared__ double s_part[2][kThreads / 64];
    const int64_t v = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
    if (v < p.num_vis)
    {
        const int64_t cell = cell_of(p, v);
        if (cell >= 0)
        {
            for (int64_t pol = 0; pol < p.P; ++pol)
            {
                const W g = grid[cell + pol];
                const W g2 = g * g;
                s1 += (double)g;
                s2 += (double)g2;
            }
        }
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
    {
        s_part[0][wave] = s1;
        s_part[1][wave] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
        double a = 0.0, b = 0.0;
        for (int w = 0; w < kThreads / 64; ++w)
        {
            a += s_part[0][w];
            b += s_part[1][w];
        }
        unsafeAtomicAdd(&sums[0], a);
        unsafeAtomicAdd(&sums[1], b);
    }
}

// out = 1 / grid (sdp_weighting.cpp:210-216).
template<typename W>
__global__ __launch_bounds__(kThreads) void k_read_uniform(WParams p,
        const W* __restrict__ grid, W* __restrict__ out)
{
    const int64_t v = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (v >= p.num_vis) return;
    const int64_t cell = cell_of(p, v);
    if (cell < 0) return;
    for (int64_t pol = 0; pol < p.P; ++pol)
        out[v * p.P + pol] = (W)(1.0 / (double)grid[cell + pol]);
}

// out = in / (1 + R grid), R = numerator / (sum2 / sum)
// (sdp_weighting.cpp:143-154, 270-279).
template<typename W>
__global__ __launch_bounds__(kThreads) void k_read_briggs(WParams p,
        const W* __restrict__ grid, const W* __restrict__ in,
        W* __restrict__ out, const double* __restrict__ sums, double numer)
{
#pragma clang fp contract(off)
    const int64_t v = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (v >= p.num_vis) return;
    const int64_t cell = cell_of(p, v);
    if (cell < 0) return;
    const double robustness = numer / (sums[1] / sums[0]);
    for (int64_t pol = 0; pol < p.P; ++pol)
    {
        const double den = 1.0 + robustness * (double)grid[cell + pol];
        out[v * p.P + pol] = (W)((double)in[v * p.P + pol] / den);
    }
}

// Argument checks of the reference (sdp_weighting.cpp:286-336), with its
// status codes; returns the metadata.
bool check_args(const sdp_Mem* uvw, const sdp_Mem* freq_hz,
        sdp_Mem* weights_grid_uv, sdp_Mem* input_weight,
        sdp_Mem* output_weight, int64_t* dims, sdp_Error* status)
{
    if (*status) return false;
    for (const sdp_Mem* w : {(const sdp_Mem*)input_weight,
            (const sdp_Mem*)output_weight})
    {
        if (*status) break;
        if (sdp_mem_num_dims(w) != 4)
        {
            *status = SDP_ERR_RUNTIME;
            SDP_LOG_ERROR("The weights array must be 4D");
            break;
        }
        if (sdp_mem_is_complex(w))
        {
            *status = SDP_ERR_DATA_TYPE;
            SDP_LOG_ERROR("The weights array cannot be complex");
            break;
        }
        for (int d = 0; d < 4; ++d) dims[d] = sdp_mem_shape_dim(w, d);
    }
    if (*status) return false;
    const sdp_MemLocation loc = sdp_mem_location(output_weight);
    // dims[] holds the output's {T, B, C, P}; the kernels index the input
    // with the same flat offsets, so it must live where the output lives
    // (the reference's GPU path fetches it with sdp_mem_gpu_buffer_const,
    // which fails with SDP_ERR_MEM_LOCATION) and have the same shape.
    sdp_mem_check_location(input_weight, loc, status);
    sdp_mem_check_shape(input_weight, 4, dims, status);
    if (*status) return false;
    if (!sdp_mem_is_floating_point(uvw) || sdp_mem_is_complex(uvw))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("The uvw array must be real-valued");
    }
    const int64_t uvw_shape[] = {dims[0], dims[1], 3};
    sdp_mem_check_shape(uvw, 3, uvw_shape, status);
    sdp_mem_check_location(uvw, loc, status);
    sdp_mem_check_c_contiguity(uvw, status);
    sdp_mem_check_location(freq_hz, loc, status);
    sdp_mem_check_location(weights_grid_uv, loc, status);
    sdp_mem_check_writeable(output_weight, status);
    sdp_mem_check_writeable(weights_grid_uv, status);
    sdp_mem_check_num_dims(weights_grid_uv, 3, status);
    if (*status) return false;
    const int64_t G = sdp_mem_shape_dim(weights_grid_uv, 0);
    sdp_mem_check_dim_size(weights_grid_uv, 1, G, status);
    if (*status) return false;
    // Types supported by the reference (sdp_weighting.cpp:341-405).
    const sdp_MemType wt = sdp_mem_type(output_weight);
    const bool ok = sdp_mem_type(uvw) == SDP_MEM_DOUBLE &&
            sdp_mem_type(freq_hz) == SDP_MEM_DOUBLE &&
            (wt == SDP_MEM_DOUBLE || wt == SDP_MEM_FLOAT) &&
            sdp_mem_type(input_weight) == wt &&
            sdp_mem_type(weights_grid_uv) == wt;
    if (!ok)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data type(s)");
        return false;
    }
    // This implementation also needs the arrays it indexes flat to be
    // C-contiguous and the polarisation / channel dimensions to agree.
    sdp_mem_check_c_contiguity(freq_hz, status);
    sdp_mem_check_c_contiguity(weights_grid_uv, status);
    sdp_mem_check_c_contiguity(input_weight, status);
    sdp_mem_check_c_contiguity(output_weight, status);
    sdp_mem_check_dim_size(weights_grid_uv, 2, dims[3], status);
    if (*status) return false;
    if (sdp_mem_shape_dim(freq_hz, 0) < dims[2])
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("freq_hz has fewer entries than weights has channels");
        return false;
    }
    if (!sdp_hip::device_available())
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("No GPU available for the weighting functions.");
        return false;
    }
    return true;
}

// Device views of the five arrays; host arrays are staged through HBM.
struct Views
{
    const double* uvw = nullptr;
    const double* freq = nullptr;
    void* grid = nullptr;
    const void* in = nullptr;
    void* out = nullptr;
    void* tmp[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    size_t bytes[5] = {0, 0, 0, 0, 0};
    bool staged = false;
};

void* stage(const sdp_Mem* m, Views& v, int k, sdp_Error* status)
{
    v.bytes[k] = (size_t)sdp_mem_num_elements(m) * sdp_mem_type_size(
            sdp_mem_type(m));
    if (*status) return nullptr;
    if (hipMalloc(&v.tmp[k], v.bytes[k] ? v.bytes[k] : 1) != hipSuccess)
    {
        *status = SDP_ERR_MEM_ALLOC_FAILURE;
        SDP_LOG_ERROR("Cannot stage %zu bytes in device memory", v.bytes[k]);
        return nullptr;
    }
    SDP_HIP_CHECK(hipMemcpy(v.tmp[k], sdp_mem_data_const(m), v.bytes[k],
            hipMemcpyHostToDevice), status);
    return v.tmp[k];
}

void open_views(const sdp_Mem* uvw, const sdp_Mem* freq, sdp_Mem* grid,
        const sdp_Mem* in, sdp_Mem* out, Views& v, sdp_Error* status)
{
    if (sdp_mem_location(out) == SDP_MEM_GPU)
    {
        v.uvw = (const double*)sdp_mem_data_const(uvw);
        v.freq = (const double*)sdp_mem_data_const(freq);
        v.grid = sdp_mem_data(grid);
        v.in = sdp_mem_data_const(in);
        v.out = sdp_mem_data(out);
        return;
    }
    v.staged = true;
    v.uvw = (const double*)stage(uvw, v, 0, status);
    v.freq = (const double*)stage(freq, v, 1, status);
    v.grid = stage(grid, v, 2, status);
    v.in = stage(in, v, 3, status);
    v.out = stage(out, v, 4, status);
}

void close_views(sdp_Mem* grid, sdp_Mem* out, Views& v, sdp_Error* status)
{
    if (!v.staged) return;
    if (!*status)
    {
        SDP_HIP_CHECK(hipMemcpy(sdp_mem_data(grid), v.tmp[2], v.bytes[2],
                hipMemcpyDeviceToHost), status);
        SDP_HIP_CHECK(hipMemcpy(sdp_mem_data(out), v.tmp[4], v.bytes[4],
                hipMemcpyDeviceToHost), status);
    }
    for (void* p : v.tmp) (void)hipFree(p);
}

template<typename W>
void run(const WParams& p, const Views& v, bool briggs, double robust_param,
        sdp_Error* status)
{
    if (p.num_vis == 0 || p.P == 0) return;
    const unsigned blocks = (unsigned)((p.num_vis + kThreads - 1) / kThreads);
    k_grid_write<W><<<blocks, kThreads>>>(p, (W*)v.grid, (const W*)v.in);
    SDP_HIP_CHECK_LAUNCH(status);
    if (!briggs)
    {
        k_read_uniform<W><<<blocks, kThreads>>>(p, (const W*)v.grid,
                (W*)v.out);
        SDP_HIP_CHECK_LAUNCH(status);
        return;
    }
    double* sums = nullptr;
    SDP_HIP_CHECK(hipMallocAsync((void**)&sums, 2 * sizeof(double), 0),
            status);
    if (*status) return;
    SDP_HIP_CHECK(hipMemsetAsync(sums, 0, 2 * sizeof(double), 0), status);
    k_grid_sums<W><<<blocks, kThreads>>>(p, (const W*)v.grid, sums);
    SDP_HIP_CHECK_LAUNCH(status);
    // robustness_calc, sdp_weighting.cpp:143-154 (host pow as the reference).
    const double numer = pow(5.0 * 1 / (pow(10.0, robust_param)), 2.0);
    k_read_briggs<W><<<blocks, kThreads>>>(p, (const W*)v.grid,
            (const W*)v.in, (W*)v.out, sums, numer);
    SDP_HIP_CHECK_LAUNCH(status);
    SDP_HIP_CHECK(hipFreeAsync(sums, 0), status);
}

void weighting(const sdp_Mem* uvw, const sdp_Mem* freq_hz, double max_abs_uv,
        bool briggs, double robust_param, sdp_Mem* grid, sdp_Mem* in,
        sdp_Mem* out, sdp_Error* status)
{
    int64_t dims[4] = {0, 0, 0, 0};
    if (!check_args(uvw, freq_hz, grid, in, out, dims, status)) return;
    WParams p;
    p.num_vis = dims[0] * dims[1] * dims[2];
    p.C = dims[2];
    p.P = dims[3];
    p.G = sdp_mem_shape_dim(grid, 0);
    p.max_abs_uv = max_abs_uv;
    Views v;
    open_views(uvw, freq_hz, grid, in, out, v, status);
    p.uvw = v.uvw;
    p.freq = v.freq;
    if (!*status)
    {
        if (sdp_mem_type(out) == SDP_MEM_DOUBLE)
            run<double>(p, v, briggs, robust_param, status);
        else
            run<float>(p, v, briggs, robust_param, status);
    }
    close_views(grid, out, v, status);
}

} // namespace

extern "C" {

void sdp_weighting_briggs(const sdp_Mem* uvw, const sdp_Mem* freq_hz,
        double max_abs_uv, const double robust_param,
        sdp_Mem* weight_grid_uv, sdp_Mem* input_weights,
        sdp_Mem* output_weights, sdp_Error* status)
{
    if (*status) return;
    weighting(uvw, freq_hz, max_abs_uv, true, robust_param, weight_grid_uv,
            input_weights, output_weights, status);
}

void sdp_weighting_uniform(const sdp_Mem* uvw, const sdp_Mem* freq_hz,
        double max_abs_uv, sdp_Mem* weight_grid_uv, sdp_Mem* input_weights,
        sdp_Mem* output_weights, sdp_Error* status)
{
    if (*status) return;
    weighting(uvw, freq_hz, max_abs_uv, false, 0.0, weight_grid_uv,
            input_weights, output_weights, status);
}

} // extern "C"
