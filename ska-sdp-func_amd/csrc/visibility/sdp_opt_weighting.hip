// MI355X-native tiled Briggs weighting (sdp_optimized_weighting,
// sdp_optimised_indexed_weighting).
//
// Replaces src/ska-sdp-func/visibility/sdp_opt_weighting.cpp / .cu of
// ska-sdp-func 1.2.2; semantics and the reference defects not carried over
// are listed in include/ska-sdp-func/visibility/sdp_opt_weighting.h.
//
// One workgroup of 512 threads (one per cell of a 32 x 16 tile, the
// reference's block) per run of the sorted arrays. Three passes over the
// run, all reading the run's positions contiguously:
//   1. cell sums W in LDS (ds_add_f64);
//   2. sw / sw2 per thread, then a wave reduction (DPP/permute shuffles)
//      and a 8-entry LDS reduction in a fixed order, so R is deterministic
//      given W;
//   3. out = w / (1 + R W[cell]).
// HBM-bound: per entry 2 positions + 1 tile code (+ index) read three
// times (the second and third from L2 for runs below a few MB), one
// weight read twice and one weight written.
#include <cmath>
#include <cstdint>

#include "ska-sdp-func/visibility/sdp_opt_weighting.h"
#include "../utility/sdp_hip.h"

namespace {

constexpr int kTileU = 32;
constexpr int kTileV = 16;
constexpr int kThreads = kTileU * kTileV;

struct OptArgs
{
    const double* uu;
    const double* vv;
    const double* weight;       // sorted (bucket) or original (indexed)
    const int* index;           // sorted_vis_index, or null (bucket)
    const int* tile;
    const int* offsets;
    int64_t top_u, top_v;
    int grid_size;
    int64_t num_out;            // elements of output_weights
    double numerator;           // (5 10^-robust)^2
    double* out;
};

// Cell of entry i inside the run's tile, or -1 (.cu:58-67).
__device__ __forceinline__ int cell_in_tile(const OptArgs& a, int64_t i,
        int64_t tile_u, int64_t tile_v)
{
    const int64_t centre = a.grid_size / 2;
    const int64_t gu = (int64_t)round(a.uu[i]) + centre - tile_u;
    const int64_t gv = (int64_t)round(a.vv[i]) + centre - tile_v;
    if (gu < 0 || gu >= kTileU || gv < 0 || gv >= kTileV) return -1;
    return (int)(gu * kTileV + gv);
}

__device__ __forceinline__ double wave_sum(double x)
{
    for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d);
    return x;
}

__global__ __launch_bounds__(kThreads) void k_opt_briggs(OptArgs a)
{
    __shared__ double cell[kThreads];
    __shared__ double part[2][kThreads / 64];
    const int tid = threadIdx.x;
    const int64_t start = a.offsets[blockIdx.x];
    const int64_t end = a.offsets[blockIdx.x + 1];
    if (end <= start) return;                        // uniform per block
    cell[tid] = 0.0;
    const int code = a.tile[start];
    const int64_t tile_u = (int64_t)(code & 32767) * kTileU + a.top_u;
    const int64_t tile_v = (int64_t)(code >> 15) * kTileV + a.top_v;
    __syncthreads();

    for (int64_t i = start + tid; i < end; i += kThreads)
    {
        const int c = cell_in_tile(a, i, tile_u, tile_v);
        if (c < 0) continue;
        const int64_t src = a.index ? (int64_t)a.index[i] : i;
        if (src < 0 || src >= a.num_out) continue;
        atomicAdd(&cell[c], a.weight[src]);
    }
    __syncthreads();

    double s1 = 0.0, s2 = 0.0;
    for (int64_t i = start + tid; i < end; i += kThreads)
    {
        const int c = cell_in_tile(a, i, tile_u, tile_v);
        if (c < 0) continue;
        const double w = cell[c];
        s1 += w;
        s2 += w * w;
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if ((tid & 63) == 0)
    {
        part[0][tid >> 6] = s1;
        part[1][tid >> 6] = s2;
    }
    __syncthreads();
    double sw = 0.0, sw2 = 0.0;
    for (int k = 0; k < kThreads / 64; ++k)
    {
        sw += part[0][k];
        sw2 += part[1][k];
    }
    const double robustness = a.numerator / (sw2 / sw);

    for (int64_t i = start + tid; i < end; i += kThreads)
    {
        const int c = cell_in_tile(a, i, tile_u, tile_v);
        if (c < 0) continue;
        const int64_t dst = a.index ? (int64_t)a.index[i] : i;
        if (dst < 0 || dst >= a.num_out) continue;
        a.out[dst] = a.weight[dst] / (1.0 + robustness * cell[c]);
    }
}

bool check_vis(const sdp_Mem* uvw, const sdp_Mem* vis, const sdp_Mem* weights,
        sdp_Error* status)
{
    // sdp_data_model_get_vis_metadata / check_uvw / check_weights
    // (.cpp:70-100).
    if (*status) return false;
    if (!sdp_mem_is_complex(vis))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("The visibility array must be complex");
        return false;
    }
    sdp_mem_check_num_dims(vis, 4, status);
    if (*status) return false;
    const int64_t T = sdp_mem_shape_dim(vis, 0), B = sdp_mem_shape_dim(vis, 1);
    const int64_t C = sdp_mem_shape_dim(vis, 2), P = sdp_mem_shape_dim(vis, 3);
    const int64_t shape_uvw[] = {T, B, 3};
    const int64_t shape_w[] = {T, B, C, P};
    sdp_mem_check_shape(uvw, 3, shape_uvw, status);
    sdp_mem_check_shape(weights, 4, shape_w, status);
    if (*status) return false;
    const sdp_MemLocation loc = sdp_mem_location(vis);
    if (sdp_mem_location(uvw) != loc || sdp_mem_location(weights) != loc)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("All arrays must be in the same memory space");
        return false;
    }
    return true;
}

// Type / location dispatch of the reference (.cpp:102-120).
bool check_types(const sdp_Mem* vis, bool doubles, sdp_Error* status)
{
    if (*status) return false;
    if (sdp_mem_location(vis) != SDP_MEM_GPU)
    {
        if (doubles)
        {
            *status = SDP_ERR_MEM_LOCATION;
            SDP_LOG_ERROR("CPU Briggs Weighting doesn't exist yet!");
        }
        else
        {
            *status = SDP_ERR_DATA_TYPE;
            SDP_LOG_ERROR("Unsupported data type(s)");
        }
        return false;
    }
    if (!doubles)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data type(s)");
        return false;
    }
    return true;
}

bool check_dev(const sdp_Mem* m, sdp_MemType t, int64_t min_elems,
        const char* what, sdp_Error* status)
{
    if (*status) return false;
    if (sdp_mem_location(m) != SDP_MEM_GPU)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("%s must be in GPU memory", what);
        return false;
    }
    if (sdp_mem_type(m) != t || !sdp_mem_is_c_contiguous(m) ||
            sdp_mem_num_elements(m) < min_elems)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("%s: wrong type, layout or length", what);
        return false;
    }
    return true;
}

void launch(OptArgs a, const sdp_Mem* sorted_uu, const sdp_Mem* sorted_vv,
        const sdp_Mem* sorted_tile, const sdp_Mem* tile_offsets,
        sdp_Mem* output_weights, double robust_param, int64_t ntiles,
        sdp_Error* status)
{
    const int64_t n = sdp_mem_num_elements(sorted_uu);
    if (!check_dev(sorted_uu, SDP_MEM_DOUBLE, 0, "sorted_uu", status) ||
            !check_dev(sorted_vv, SDP_MEM_DOUBLE, n, "sorted_vv", status) ||
            !check_dev(sorted_tile, SDP_MEM_INT, n, "sorted_tile", status) ||
            !check_dev(tile_offsets, SDP_MEM_INT, ntiles + 1, "tile_offsets",
                    status) ||
            !check_dev(output_weights, SDP_MEM_DOUBLE, 0, "output_weights",
                    status))
        return;
    sdp_mem_check_writeable(output_weights, status);
    if (*status) return;
    // Runs must lie inside the sorted arrays: offsets are caller data.
    if (ntiles > 1)
    {
        int* h = new int[ntiles + 1];
        SDP_HIP_CHECK(hipMemcpy(h, sdp_mem_data_const(tile_offsets),
                (ntiles + 1) * sizeof(int), hipMemcpyDeviceToHost), status);
        for (int64_t k = 0; k + 1 < ntiles && !*status; ++k)
            if (h[k + 1] > h[k] && (h[k] < 0 || h[k + 1] > n))
            {
                *status = SDP_ERR_INVALID_ARGUMENT;
                SDP_LOG_ERROR("tile_offsets run %lld [%d, %d) is outside "
                        "the %lld sorted entries", (long long)k, h[k],
                        h[k + 1], (long long)n);
            }
        delete[] h;
    }
    if (*status || ntiles < 2) return;
    a.uu = (const double*)sdp_mem_data_const(sorted_uu);
    a.vv = (const double*)sdp_mem_data_const(sorted_vv);
    a.tile = (const int*)sdp_mem_data_const(sorted_tile);
    a.offsets = (const int*)sdp_mem_data_const(tile_offsets);
    a.num_out = sdp_mem_num_elements(output_weights);
    a.numerator = pow(5.0 * 1 / (pow(10.0, robust_param)), 2.0);
    a.out = (double*)sdp_mem_data(output_weights);
    hipLaunchKernelGGL(k_opt_briggs, dim3((unsigned int)(ntiles - 1)),
            dim3(kThreads), 0, 0, a);
    SDP_HIP_CHECK_LAUNCH(status);
}

OptArgs geometry(int grid_size, int64_t* ntiles)
{
    // .cpp:47-58
    const int64_t centre = grid_size / 2;
    OptArgs a = {};
    a.grid_size = grid_size;
    a.top_u = centre - (centre / kTileU) * kTileU - kTileU / 2;
    a.top_v = centre - (centre / kTileV) * kTileV - kTileV / 2;
    *ntiles = ((grid_size + kTileU - 1) / kTileU) *
            (int64_t)((grid_size + kTileV - 1) / kTileV);
    return a;
}

} // namespace

extern "C" {

void sdp_optimized_weighting(const sdp_Mem* uvw, const sdp_Mem* freqs,
        const sdp_Mem* vis, const sdp_Mem* weights, const double robust_param,
        const int grid_size, const int64_t support, sdp_Mem* sorted_uu,
        sdp_Mem* sorted_vv, sdp_Mem* sorted_weight, sdp_Mem* sorted_tile,
        sdp_Mem* tile_offsets, sdp_Mem* num_points_in_tiles,
        sdp_Mem* output_weights, sdp_Error* status)
{
    (void)support;
    (void)num_points_in_tiles;
    if (*status) return;
    if (!check_vis(uvw, vis, weights, status)) return;
    const bool doubles = sdp_mem_type(uvw) == SDP_MEM_DOUBLE &&
            sdp_mem_type(weights) == SDP_MEM_DOUBLE &&
            sdp_mem_type(freqs) == SDP_MEM_DOUBLE;
    if (!check_types(vis, doubles, status)) return;
    if (grid_size < 1)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("grid_size must be positive");
        return;
    }
    int64_t ntiles = 0;
    OptArgs a = geometry(grid_size, &ntiles);
    const int64_t n = sdp_mem_num_elements(sorted_uu);
    if (!check_dev(sorted_weight, SDP_MEM_DOUBLE, n, "sorted_weight", status))
        return;
    if (sdp_mem_num_elements(output_weights) < n)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("output_weights is shorter than the sorted arrays");
        return;
    }
    a.weight = (const double*)sdp_mem_data_const(sorted_weight);
    a.index = nullptr;
    launch(a, sorted_uu, sorted_vv, sorted_tile, tile_offsets,
            output_weights, robust_param, ntiles, status);
}

void sdp_optimised_indexed_weighting(const sdp_Mem* uvw, const sdp_Mem* vis,
        const sdp_Mem* weights, const double robust_param, const int grid_size,
        const double cell_size_rad, const int64_t support,
        const int* num_visibilites, sdp_Mem* sorted_tile, sdp_Mem* sorted_uu,
        sdp_Mem* sorted_vv, sdp_Mem* sorted_vis_index, sdp_Mem* tile_offsets,
        sdp_Mem* num_points_in_tiles, sdp_Mem* output_weights,
        sdp_Error* status)
{
    (void)cell_size_rad;
    (void)support;
    (void)num_visibilites;
    (void)num_points_in_tiles;
    if (*status) return;
    if (!check_vis(uvw, vis, weights, status)) return;
    const bool doubles = sdp_mem_type(uvw) == SDP_MEM_DOUBLE &&
            sdp_mem_type(weights) == SDP_MEM_DOUBLE;
    if (!check_types(vis, doubles, status)) return;
    if (grid_size < 1)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("grid_size must be positive");
        return;
    }
    int64_t ntiles = 0;
    OptArgs a = geometry(grid_size, &ntiles);
    const int64_t n = sdp_mem_num_elements(sorted_uu);
    if (!check_dev(sorted_vis_index, SDP_MEM_INT, n, "sorted_vis_index",
            status))
        return;
    if (!check_dev(weights, SDP_MEM_DOUBLE, 0, "weights", status)) return;
    if (sdp_mem_num_elements(output_weights) !=
            sdp_mem_num_elements(weights))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("output_weights must have the shape of weights");
        return;
    }
    a.weight = (const double*)sdp_mem_data_const(weights);
    a.index = (const int*)sdp_mem_data_const(sorted_vis_index);
    launch(a, sorted_uu, sorted_vv, sorted_tile, tile_offsets,
            output_weights, robust_param, ntiles, status);
}

} // extern "C"
