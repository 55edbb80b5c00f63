// MI355X-native tiling and bucket sort of visibilities
// (sdp_count_and_prefix_sum, sdp_bucket_sort, sdp_tiled_indexing).
//
// Replaces src/ska-sdp-func/visibility/sdp_tiled_functions.cpp / .cu of
// ska-sdp-func 1.2.2 with the reference GPU kernels' tile arithmetic
// (sdp_tiled_functions.cu:63-291) and a deterministic order. The reference
// appends entries with one atomic cursor per tile, so the order inside a
// tile depends on scheduling; here the sort is a stable radix sort:
//   1. k_tile_count: per visibility, its tiles (per-tile counts, skipped
//      count, entries per visibility);
//   2. exclusive scans (hipCUB) of entries per visibility and of tile counts;
//   3. k_tile_emit: (tile, visibility) pairs in visibility order;
//   4. hipCUB DeviceRadixSort (stable) on the tile key, so each tile lists
//      its visibilities in (time, baseline, channel) order;
//   5. k_tile_write: entry j of tile k goes to the caller's
//      tile_offsets[k] + (its rank in tile k), and tile_offsets[k] advances
//      by the tile's count, as the reference cursors do.
// Integer / HBM-bound work: a few passes over visibilities and entries.
#include <cmath>
#include <cstdint>

#include <hipcub/hipcub.hpp>

#include "ska-sdp-func/visibility/sdp_tiled_functions.h"
#include "../utility/sdp_hip.h"

namespace {

constexpr double kC0 = 299792458.0;
constexpr int kThreads = 256;

struct TileGeom
{
    int64_t T, B, C, nvis;
    int grid;
    int64_t support;
    float inv_tu, inv_tv;
    int64_t ntu, ntiles, top_u, top_v;
    double grid_scale;
};

TileGeom make_geom(int grid, int64_t tu, int64_t tv, double cell,
        int64_t support, int64_t T, int64_t B, int64_t C)
{
    // sdp_tiled_functions.cpp:331-342.
    TileGeom g;
    g.T = T;
    g.B = B;
    g.C = C;
    g.nvis = T * B * C;
    g.grid = grid;
    g.support = support;
    const int64_t centre = grid / 2;
    g.inv_tu = (float)(1.0 / tu);
    g.inv_tv = (float)(1.0 / tv);
    g.ntu = (grid + tu - 1) / tu;
    g.ntiles = g.ntu * ((grid + tv - 1) / tv);
    g.top_u = centre - (centre / tu) * tu - tu / 2;
    g.top_v = centre - (centre / tv) * tv - tv / 2;
    g.grid_scale = grid * cell;
    return g;
}

struct Range
{
    int u0, u1, v0, v1;   // tiles [u0, u1) x [v0, v1)
};

// Position and tile range of visibility v (.cu:91-114); false if skipped.
template<typename U>
__device__ __forceinline__ bool tiles_of(const TileGeom& g,
        const U* __restrict__ uvw, const U* __restrict__ freq, int64_t v,
        U& pos_u, U& pos_v, Range& r)
{
#pragma clang fp contract(off)
    const int64_t tb = v / g.C, c = v - tb * g.C;
    const U inv_wl = (U)((double)freq[c] / kC0);
    pos_u = (U)((double)(uvw[3 * tb] * inv_wl) * g.grid_scale);
    pos_v = (U)((double)(uvw[3 * tb + 1] * inv_wl) * g.grid_scale);
    const int64_t centre = g.grid / 2;
    const int64_t gu = (int64_t)round(pos_u) + centre;
    const int64_t gv = (int64_t)round(pos_v) + centre;
    if (!(gu + g.support < g.grid && gu - g.support >= 0 &&
            gv + g.support < g.grid && gv - g.support >= 0))
        return false;
    const int rel_u = (int)(gu - g.top_u), rel_v = (int)(gv - g.top_v);
    const float u1 = (float)(rel_u - g.support) * g.inv_tu;
    const float u2 = (float)(rel_u + g.support + 1) * g.inv_tu;
    const float v1 = (float)(rel_v - g.support) * g.inv_tv;
    const float v2 = (float)(rel_v + g.support + 1) * g.inv_tv;
    r.u0 = (int)floorf(u1);
    r.u1 = (int)ceilf(u2);
    r.v0 = (int)floorf(v1);
    r.v1 = (int)ceilf(v2);
    return true;
}

__device__ __forceinline__ bool tile_ok(const TileGeom& g, int pu, int pv,
        int64_t& idx)
{
    idx = (int64_t)pu + (int64_t)pv * g.ntu;
    return idx >= 0 && idx < g.ntiles;
}

template<typename U>
__global__ void k_tile_count(TileGeom g, const U* __restrict__ uvw,
        const U* __restrict__ freq, int* __restrict__ counts,
        int* __restrict__ skipped, int* __restrict__ nent)
{
    const int64_t v = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (v >= g.nvis) return;
    U pu, pv;
    Range r;
    int n = 0;
    if (!tiles_of(g, uvw, freq, v, pu, pv, r))
    {
        atomicAdd(skipped, 1);
    }
    else
    {
        for (int b = r.v0; b < r.v1; ++b)
            for (int a = r.u0; a < r.u1; ++a)
            {
                int64_t idx;
                if (!tile_ok(g, a, b, idx)) continue;
                atomicAdd(&counts[idx], 1);
                ++n;
            }
    }
    if (nent) nent[v] = n;
}

template<typename U>
__global__ void k_tile_emit(TileGeom g, const U* __restrict__ uvw,
        const U* __restrict__ freq, const int* __restrict__ eoff,
        int* __restrict__ keys, int* __restrict__ vals)
{
    const int64_t v = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (v >= g.nvis) return;
    U pu, pv;
    Range r;
    if (!tiles_of(g, uvw, freq, v, pu, pv, r)) return;
    int o = eoff[v];
    for (int b = r.v0; b < r.v1; ++b)
        for (int a = r.u0; a < r.u1; ++a)
        {
            int64_t idx;
            if (!tile_ok(g, a, b, idx)) continue;
            keys[o] = (int)idx;
            vals[o] = (int)v;
            ++o;
        }
}

template<typename U>
struct SortOut
{
    U* uu;
    U* vv;
    U* vis;          // bucket sort: element (t, b, c) of vis read as U
    U* weight;
    int* tile;
    int* vis_index;  // tiled indexing
    int64_t cap;     // output length
};

template<typename U>
__global__ void k_tile_write(TileGeom g, const U* __restrict__ uvw,
        const U* __restrict__ freq, const U* __restrict__ vis_as_u,
        const U* __restrict__ weight, const int* __restrict__ keys,
        const int* __restrict__ vals, int64_t n_entries,
        const int* __restrict__ tstart, const int* __restrict__ offsets,
        SortOut<U> o)
{
    const int64_t j = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (j >= n_entries) return;
    const int k = keys[j], v = vals[j];
    const int64_t pos = (int64_t)offsets[k] + (j - tstart[k]);
    if (pos < 0 || pos >= o.cap) return;
    U pu, pv;
    Range r;
    tiles_of(g, uvw, freq, v, pu, pv, r);
    // The (pu, pv) of this entry: the first in the visibility's range whose
    // flat index is k (a u range past the grid edge aliases into the next
    // row, and the reference stores the unwrapped pair).
    int code = (int)(k / g.ntu) * 32768 + (int)(k % g.ntu);
    for (int b = r.v0; b < r.v1; ++b)
        for (int a = r.u0; a < r.u1; ++a)
            if ((int64_t)a + (int64_t)b * g.ntu == k)
            {
                code = b * 32768 + a;
                b = r.v1;
                break;
            }
    o.uu[pos] = pu;
    o.vv[pos] = pv;
    o.tile[pos] = code;
    if (o.vis) o.vis[pos] = vis_as_u[v];
    if (o.weight) o.weight[pos] = weight[v];
    if (o.vis_index) o.vis_index[pos] = v;
}

// Sets *bad when some tile's run [offsets[k], offsets[k] + counts[k]) does
// not lie inside the caller's sorted arrays [0, cap).
__global__ void k_check_fit(const int* __restrict__ offsets,
        const int* __restrict__ counts, int64_t ntiles, int64_t cap,
        int* __restrict__ bad)
{
    const int64_t k = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (k >= ntiles || counts[k] == 0) return;
    const int64_t lo = offsets[k], hi = lo + counts[k];
    if (lo < 0 || hi > cap) *bad = 1;
}

__global__ void k_advance(int* __restrict__ offsets,
        const int* __restrict__ counts, int64_t ntiles)
{
    const int64_t k = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (k < ntiles) offsets[k] += counts[k];
}

unsigned int blocks(int64_t n)
{
    return (unsigned int)((n + kThreads - 1) / kThreads);
}

bool on_gpu(const sdp_Mem* m, sdp_Error* status)
{
    if (sdp_mem_location(m) != SDP_MEM_GPU)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("The tiled functions need all arrays in GPU memory");
        return false;
    }
    return true;
}

bool check_int(const sdp_Mem* m, int64_t min_elems, sdp_Error* status)
{
    if (*status) return false;
    if (!on_gpu(m, status)) return false;
    if (sdp_mem_type(m) != SDP_MEM_INT || !sdp_mem_is_c_contiguous(m) ||
            sdp_mem_num_elements(m) < min_elems)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Tile arrays must be contiguous int32 of the tile count");
        return false;
    }
    return true;
}

// Visibility metadata (sdp_data_model_get_vis_metadata) and uvw shape.
bool vis_dims(const sdp_Mem* vis, const sdp_Mem* uvw, int64_t* T, int64_t* B,
        int64_t* C, int64_t* P, sdp_Error* status)
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
    *T = sdp_mem_shape_dim(vis, 0);
    *B = sdp_mem_shape_dim(vis, 1);
    *C = sdp_mem_shape_dim(vis, 2);
    *P = sdp_mem_shape_dim(vis, 3);
    const int64_t shape_uvw[] = {*T, *B, 3};
    sdp_mem_check_shape(uvw, 3, shape_uvw, status);
    return !*status;
}

bool real_pair(const sdp_Mem* uvw, const sdp_Mem* freqs, bool* dbl,
        sdp_Error* status)
{
    if (*status) return false;
    const sdp_MemType t = sdp_mem_type(uvw);
    if ((t != SDP_MEM_DOUBLE && t != SDP_MEM_FLOAT) ||
            sdp_mem_type(freqs) != t)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data type(s)");
        return false;
    }
    *dbl = t == SDP_MEM_DOUBLE;
    sdp_mem_check_c_contiguity(uvw, status);
    sdp_mem_check_c_contiguity(freqs, status);
    if (*status) return false;
    return on_gpu(uvw, status) && on_gpu(freqs, status);
}

// Shared body of bucket sort and tiled indexing.
template<typename U>
void sort_tiles(const TileGeom& g, const U* uvw, const U* freq,
        const U* vis_as_u, const U* weight, int* offsets, SortOut<U> o,
        sdp_Error* status)
{
    if (*status || g.nvis == 0) return;
    int *counts = nullptr, *nent = nullptr, *eoff = nullptr, *tstart = nullptr;
    int *keys = nullptr, *vals = nullptr, *keys2 = nullptr, *vals2 = nullptr;
    int* skipped = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0, b1 = 0, b2 = 0, b3 = 0;
    const int64_t nt = g.ntiles;
    auto alloc = [&](int** p, int64_t n) {
        if (!*status && hipMalloc(p, (size_t)(n > 0 ? n : 1) * sizeof(int)) !=
                hipSuccess)
        {
            *status = SDP_ERR_MEM_ALLOC_FAILURE;
            SDP_LOG_ERROR("Unable to allocate tiling scratch");
        }
    };
    alloc(&counts, nt + 1);
    alloc(&nent, g.nvis + 1);
    alloc(&eoff, g.nvis + 1);
    alloc(&tstart, nt + 1);
    alloc(&skipped, 1);
    if (!*status)
    {
        SDP_HIP_CHECK(hipMemset(counts, 0, (nt + 1) * sizeof(int)), status);
        SDP_HIP_CHECK(hipMemset(nent, 0, (g.nvis + 1) * sizeof(int)), status);
        k_tile_count<U><<<blocks(g.nvis), kThreads>>>(g, uvw, freq, counts,
                skipped, nent);
        SDP_HIP_CHECK_LAUNCH(status);
        SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, b1, nent,
                eoff, (int)(g.nvis + 1)), status);
        SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, b2, counts,
                tstart, (int)(nt + 1)), status);
    }
    int n_entries = 0;
    if (!*status)
    {
        tmp_bytes = b1 > b2 ? b1 : b2;
        if (hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 1) != hipSuccess)
            *status = SDP_ERR_MEM_ALLOC_FAILURE;
    }
    if (!*status)
    {
        SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, b1, nent, eoff,
                (int)(g.nvis + 1)), status);
        SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, b2, counts,
                tstart, (int)(nt + 1)), status);
        SDP_HIP_CHECK(hipMemcpy(&n_entries, eoff + g.nvis, sizeof(int),
                hipMemcpyDeviceToHost), status);
    }
    // The caller's offsets plus this call's per-tile counts must fit the
    // sorted arrays: refuse rather than truncate (a truncated write would
    // leave the advanced cursors inconsistent with what was stored).
    if (!*status && (int64_t)n_entries > o.cap)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Sorted arrays hold %lld entries, %d needed",
                (long long)o.cap, n_entries);
    }
    if (!*status && n_entries > 0)
    {
        int bad = 0;
        SDP_HIP_CHECK(hipMemset(skipped, 0, sizeof(int)), status);
        k_check_fit<<<blocks(nt), kThreads>>>(offsets, counts, nt, o.cap,
                skipped);
        SDP_HIP_CHECK_LAUNCH(status);
        SDP_HIP_CHECK(hipMemcpy(&bad, skipped, sizeof(int),
                hipMemcpyDeviceToHost), status);
        if (!*status && bad)
        {
            *status = SDP_ERR_INVALID_ARGUMENT;
            SDP_LOG_ERROR("tile_offsets + tile counts run past the sorted "
                    "arrays (%lld entries)", (long long)o.cap);
        }
    }
    if (*status)
    {
        int* bufs[] = {counts, nent, eoff, tstart, skipped};
        for (int* p : bufs) (void)hipFree(p);
        (void)hipFree(tmp);
        return;
    }
    alloc(&keys, n_entries);
    alloc(&vals, n_entries);
    alloc(&keys2, n_entries);
    alloc(&vals2, n_entries);
    int end_bit = 1;
    while (end_bit < 31 && ((int64_t)1 << end_bit) < nt) ++end_bit;
    if (!*status && n_entries > 0)
    {
        k_tile_emit<U><<<blocks(g.nvis), kThreads>>>(g, uvw, freq, eoff,
                keys, vals);
        SDP_HIP_CHECK_LAUNCH(status);
        SDP_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, b3, keys,
                keys2, vals, vals2, n_entries, 0, end_bit), status);
        void* tmp2 = nullptr;
        if (!*status && hipMalloc(&tmp2, b3 ? b3 : 1) != hipSuccess)
            *status = SDP_ERR_MEM_ALLOC_FAILURE;
        if (!*status)
            SDP_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp2, b3, keys,
                    keys2, vals, vals2, n_entries, 0, end_bit), status);
        if (!*status)
        {
            k_tile_write<U><<<blocks(n_entries), kThreads>>>(g, uvw, freq,
                    vis_as_u, weight, keys2, vals2, n_entries, tstart,
                    offsets, o);
            SDP_HIP_CHECK_LAUNCH(status);
        }
        SDP_HIP_CHECK(hipDeviceSynchronize(), status);
        (void)hipFree(tmp2);
    }
    if (!*status)
    {
        k_advance<<<blocks(nt), kThreads>>>(offsets, counts, nt);
        SDP_HIP_CHECK_LAUNCH(status);
        SDP_HIP_CHECK(hipDeviceSynchronize(), status);
    }
    int* bufs[] = {counts, nent, eoff, tstart, keys, vals, keys2, vals2,
            skipped};
    for (int* p : bufs) (void)hipFree(p);
    (void)hipFree(tmp);
}

template<typename U>
SortOut<U> out_arrays(sdp_Mem* uu, sdp_Mem* vv, sdp_Mem* tile, int64_t cap)
{
    SortOut<U> o;
    o.uu = (U*)sdp_mem_data(uu);
    o.vv = (U*)sdp_mem_data(vv);
    o.tile = (int*)sdp_mem_data(tile);
    o.vis = nullptr;
    o.weight = nullptr;
    o.vis_index = nullptr;
    o.cap = cap;
    return o;
}

bool check_sorted(sdp_Mem* m, sdp_MemType t, int64_t cap, sdp_Error* status)
{
    if (*status) return false;
    if (!on_gpu(m, status)) return false;
    sdp_mem_check_writeable(m, status);
    if (*status) return false;
    if (sdp_mem_type(m) != t || !sdp_mem_is_c_contiguous(m) ||
            sdp_mem_num_elements(m) < cap)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Sorted output arrays must be contiguous, of equal "
                "length and of the uvw precision (int32 for tiles and "
                "indices)");
        return false;
    }
    return true;
}

void clear_all(sdp_Mem* const* arrays, int n, sdp_Error* status)
{
    // Outputs cleared first, as the reference (.cpp:514-518, :733-736).
    for (int k = 0; k < n && !*status; ++k)
    {
        const size_t bytes = (size_t)sdp_mem_num_elements(arrays[k]) *
                sdp_mem_type_size(sdp_mem_type(arrays[k]));
        SDP_HIP_CHECK(hipMemset(sdp_mem_data(arrays[k]), 0, bytes), status);
    }
}

} // namespace

extern "C" {

void sdp_count_and_prefix_sum(const sdp_Mem* uvw, const sdp_Mem* freqs,
        const sdp_Mem* vis, const int grid_size, const int64_t tile_size_u,
        const int64_t tile_size_v, const double cell_size_rad,
        const int64_t support, int* num_visibilites, sdp_Mem* tile_offsets,
        sdp_Mem* num_points_in_tiles, sdp_Mem* num_skipped, sdp_Error* status)
{
    if (*status) return;
    int64_t T = 0, B = 0, C = 0, P = 0;
    bool dbl = false;
    if (!vis_dims(vis, uvw, &T, &B, &C, &P, status)) return;
    if (!real_pair(uvw, freqs, &dbl, status)) return;
    if (tile_size_u < 1 || tile_size_v < 1 || grid_size < 1)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Grid and tile sizes must be positive");
        return;
    }
    const TileGeom g = make_geom(grid_size, tile_size_u, tile_size_v,
            cell_size_rad, support, T, B, C);
    if (!check_int(tile_offsets, g.ntiles + 1, status) ||
            !check_int(num_points_in_tiles, g.ntiles, status) ||
            !check_int(num_skipped, 1, status))
        return;
    int* counts = (int*)sdp_mem_data(num_points_in_tiles);
    int* offsets = (int*)sdp_mem_data(tile_offsets);
    int* skipped = (int*)sdp_mem_data(num_skipped);
    // Outputs cleared first (.cpp:318-321).
    SDP_HIP_CHECK(hipMemset(offsets, 0, (g.ntiles + 1) * sizeof(int)), status);
    SDP_HIP_CHECK(hipMemset(counts, 0, g.ntiles * sizeof(int)), status);
    SDP_HIP_CHECK(hipMemset(skipped, 0, sizeof(int)), status);
    if (*status) return;
    if (g.nvis > 0)
    {
        if (dbl)
            k_tile_count<double><<<blocks(g.nvis), kThreads>>>(g,
                    (const double*)sdp_mem_data_const(uvw),
                    (const double*)sdp_mem_data_const(freqs), counts,
                    skipped, nullptr);
        else
            k_tile_count<float><<<blocks(g.nvis), kThreads>>>(g,
                    (const float*)sdp_mem_data_const(uvw),
                    (const float*)sdp_mem_data_const(freqs), counts,
                    skipped, nullptr);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    // offsets[0..ntiles] = exclusive prefix of counts with a trailing 0, so
    // offsets[ntiles] is the total (.cpp:106-122).
    int* ext = nullptr;
    void* tmp = nullptr;
    size_t bytes = 0;
    if (!*status && hipMalloc(&ext, (g.ntiles + 1) * sizeof(int)) != hipSuccess)
        *status = SDP_ERR_MEM_ALLOC_FAILURE;
    if (!*status)
    {
        SDP_HIP_CHECK(hipMemset(ext, 0, (g.ntiles + 1) * sizeof(int)), status);
        SDP_HIP_CHECK(hipMemcpy(ext, counts, g.ntiles * sizeof(int),
                hipMemcpyDeviceToDevice), status);
        SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, ext,
                offsets, (int)(g.ntiles + 1)), status);
        if (!*status && hipMalloc(&tmp, bytes ? bytes : 1) != hipSuccess)
            *status = SDP_ERR_MEM_ALLOC_FAILURE;
        if (!*status)
            SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, bytes, ext,
                    offsets, (int)(g.ntiles + 1)), status);
    }
    int total = 0;
    if (!*status)
        SDP_HIP_CHECK(hipMemcpy(&total, offsets + g.ntiles, sizeof(int),
                hipMemcpyDeviceToHost), status);
    if (!*status && num_visibilites) *num_visibilites = total;
    (void)hipFree(ext);
    (void)hipFree(tmp);
}

void sdp_bucket_sort(const sdp_Mem* uvw, const sdp_Mem* freqs,
        const sdp_Mem* vis, const sdp_Mem* weights, const int grid_size,
        const int64_t tile_size_u, const int64_t tile_size_v,
        const double cell_size_rad, const int64_t support, sdp_Mem* sorted_uu,
        sdp_Mem* sorted_vv, sdp_Mem* sorted_weight, sdp_Mem* sorted_tile,
        sdp_Mem* sorted_vis, sdp_Mem* tile_offsets, sdp_Error* status)
{
    if (*status) return;
    int64_t T = 0, B = 0, C = 0, P = 0;
    bool dbl = false;
    if (!vis_dims(vis, uvw, &T, &B, &C, &P, status)) return;
    const int64_t shape_w[] = {T, B, C, P};
    sdp_mem_check_shape(weights, 4, shape_w, status);
    if (!real_pair(uvw, freqs, &dbl, status)) return;
    const sdp_MemType ut = sdp_mem_type(uvw);
    if (sdp_mem_type(weights) != ut)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data type(s)");
        return;
    }
    if (!on_gpu(vis, status) || !on_gpu(weights, status)) return;
    if (tile_size_u < 1 || tile_size_v < 1 || grid_size < 1)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Grid and tile sizes must be positive");
        return;
    }
    const TileGeom g = make_geom(grid_size, tile_size_u, tile_size_v,
            cell_size_rad, support, T, B, C);
    const int64_t cap = sdp_mem_num_elements(sorted_uu);
    if (!check_sorted(sorted_uu, ut, cap, status) ||
            !check_sorted(sorted_vv, ut, cap, status) ||
            !check_sorted(sorted_weight, ut, cap, status) ||
            !check_sorted(sorted_vis, ut, cap, status) ||
            !check_sorted(sorted_tile, SDP_MEM_INT, cap, status) ||
            !check_int(tile_offsets, g.ntiles + 1, status))
        return;
    sdp_Mem* const outs[] = {sorted_uu, sorted_vv, sorted_weight, sorted_tile,
            sorted_vis};
    clear_all(outs, 5, status);
    int* offsets = (int*)sdp_mem_data(tile_offsets);
    if (*status) return;
    if (dbl)
    {
        SortOut<double> o = out_arrays<double>(sorted_uu, sorted_vv,
                sorted_tile, cap);
        o.vis = (double*)sdp_mem_data(sorted_vis);
        o.weight = (double*)sdp_mem_data(sorted_weight);
        sort_tiles<double>(g, (const double*)sdp_mem_data_const(uvw),
                (const double*)sdp_mem_data_const(freqs),
                (const double*)sdp_mem_data_const(vis),
                (const double*)sdp_mem_data_const(weights), offsets, o,
                status);
    }
    else
    {
        SortOut<float> o = out_arrays<float>(sorted_uu, sorted_vv,
                sorted_tile, cap);
        o.vis = (float*)sdp_mem_data(sorted_vis);
        o.weight = (float*)sdp_mem_data(sorted_weight);
        sort_tiles<float>(g, (const float*)sdp_mem_data_const(uvw),
                (const float*)sdp_mem_data_const(freqs),
                (const float*)sdp_mem_data_const(vis),
                (const float*)sdp_mem_data_const(weights), offsets, o,
                status);
    }
}

void sdp_tiled_indexing(const sdp_Mem* uvw, const sdp_Mem* freqs,
        const int grid_size, const int64_t tile_size_u,
        const int64_t tile_size_v, const double cell_size_rad,
        const int64_t support, const int64_t num_channels,
        const int64_t num_baselines, const int64_t num_times,
        sdp_Mem* sorted_tile, sdp_Mem* sorted_uu, sdp_Mem* sorted_vv,
        sdp_Mem* sorted_vis_index, sdp_Mem* tile_offsets, sdp_Error* status)
{
    if (*status) return;
    const int64_t shape_uvw[] = {num_times, num_baselines, 3};
    sdp_mem_check_shape(uvw, 3, shape_uvw, status);
    bool dbl = false;
    if (!real_pair(uvw, freqs, &dbl, status)) return;
    if (sdp_mem_num_elements(freqs) < num_channels)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Fewer frequencies than channels");
        return;
    }
    if (tile_size_u < 1 || tile_size_v < 1 || grid_size < 1)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Grid and tile sizes must be positive");
        return;
    }
    const TileGeom g = make_geom(grid_size, tile_size_u, tile_size_v,
            cell_size_rad, support, num_times, num_baselines, num_channels);
    const sdp_MemType ut = sdp_mem_type(uvw);
    const int64_t cap = sdp_mem_num_elements(sorted_uu);
    if (!check_sorted(sorted_uu, ut, cap, status) ||
            !check_sorted(sorted_vv, ut, cap, status) ||
            !check_sorted(sorted_tile, SDP_MEM_INT, cap, status) ||
            !check_sorted(sorted_vis_index, SDP_MEM_INT, cap, status) ||
            !check_int(tile_offsets, g.ntiles + 1, status))
        return;
    sdp_Mem* const outs[] = {sorted_tile, sorted_vis_index, sorted_vv,
            sorted_uu};
    clear_all(outs, 4, status);
    int* offsets = (int*)sdp_mem_data(tile_offsets);
    if (*status) return;
    if (dbl)
    {
        SortOut<double> o = out_arrays<double>(sorted_uu, sorted_vv,
                sorted_tile, cap);
        o.vis_index = (int*)sdp_mem_data(sorted_vis_index);
        sort_tiles<double>(g, (const double*)sdp_mem_data_const(uvw),
                (const double*)sdp_mem_data_const(freqs), nullptr, nullptr,
                offsets, o, status);
    }
    else
    {
        SortOut<float> o = out_arrays<float>(sorted_uu, sorted_vv,
                sorted_tile, cap);
        o.vis_index = (int*)sdp_mem_data(sorted_vis_index);
        sort_tiles<float>(g, (const float*)sdp_mem_data_const(uvw),
                (const float*)sdp_mem_data_const(freqs), nullptr, nullptr,
                offsets, o, status);
    }
}

} // extern "C"
