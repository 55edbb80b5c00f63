// MI355X-native ES-FFT (de)gridder: plan, argument checks and driver.
//
// Replaces src/ska-sdp-func/grid_data/sdp_gridder_uvw_es_fft.cpp of the
// reference. Argument checks and their error codes/messages follow
// sdp_gridder_check_buffers (:72-243) and check_parameters (:246-262); the
// plan geometry (w-planes, scales, correction tables) follows create_plan
// (:305-424). The compute path is different: per w-plane, visibilities are
// bucketed by grid tile and scattered through LDS (es_kernels.hip), the FFT
// is rocFFT with a plan cached in the gridder plan, and the image-plane
// steps are fused (2-D: one kernel for screen + correction).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "ska-sdp-func/grid_data/sdp_gridder_uvw_es_fft.h"
#include "es_kernels.h"
#include "es_params.h"
#include "../fft/fft2d.h"
#include "es_fft.h"
#include "../utility/sdp_hip.h"

struct sdp_GridderUvwEsFft
{
    double pixsize_x_rad;
    double pixsize_y_rad;
    double epsilon;
    int do_wstacking;
    int num_rows;
    int num_chan;
    int image_size;
    int grid_size;
    int support;
    double beta;          // full beta (table beta * support)
    float tap_poly[sdp_es::kTapPolyPairs][sdp_es::kTapPolyDeg + 1][2];
    int tap_poly_ok;      // f32 plan with W = 8: polynomial interior taps
    double pixel_size;
    double uv_scale;
    double min_plane_w;
    double max_plane_w;
    double min_abs_w;
    double max_abs_w;
    int num_total_w_grids;
    double w_scale;
    double inv_w_scale;
    double inv_w_range;
    double conv_corr_norm_factor;
    int is_double;
    int64_t max_batch_vis;      // caller's cap on visibilities per batch

    // Device state.
    void* grid;                 // G x G complex plane
    void* grid_x[2];            // further planes of a 3-D multi-plane pass
    void* tables;               // conv_corr | quad kernel | nodes | weights
    int ntiles;
    int ncoarse;
    int ncbins;
    int nbins;
    int sshift, nsuper, nsbins, tstride;    // super bins (bucketing level 1)
    sdp_es::BucketScratch scratch;
    sdp_fft::Plan2D* fft;       // rocFFT (f64, or grids es_fft does not take)
    int fused_fft;              // f32 power-of-two grid: pruned fused passes
    sdp_es::FftTwiddles fft_tw;
    hipStream_t stream;

    // Timing.
    int timing;
    hipEvent_t ev[5];
    double acc_ms[5];
    int have_timing;
};

namespace {

const char* kMsgLocation = "Memory location mismatch.";

void check_buffers(const sdp_Mem* uvw, const sdp_Mem* freq_hz,
        const sdp_Mem* vis, const sdp_Mem* weight, const sdp_Mem* dirty_image,
        bool do_degridding, sdp_Error* status)
{
    if (*status) return;
    // dirty_image may be NULL (split-gridding API): its checks are skipped.
    if (!dirty_image) dirty_image = weight;
    const bool have_image = dirty_image != weight;
    const sdp_MemLocation loc = sdp_mem_location(uvw);
    if (loc != sdp_mem_location(freq_hz) || loc != sdp_mem_location(vis) ||
            loc != sdp_mem_location(weight) ||
            loc != sdp_mem_location(dirty_image))
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("%s", kMsgLocation);
        return;
    }
    struct { const sdp_Mem* m; bool complex; const char* msg; } kinds[] = {
        {uvw, false, "uvw values must be real."},
        {freq_hz, false, "Frequency values must be real."},
        {vis, true, "Visibility values must be complex."},
        {weight, false, "Weight values must be real."},
        {dirty_image, false, "Dirty image must be real"},
    };
    for (const auto& k : kinds)
    {
        if ((sdp_mem_is_complex(k.m) != 0) != k.complex)
        {
            *status = SDP_ERR_DATA_TYPE;
            SDP_LOG_ERROR("%s", k.msg);
            return;
        }
    }
    const int64_t num_vis = sdp_mem_shape_dim(vis, 0);
    const int64_t num_chan = sdp_mem_shape_dim(vis, 1);
    if (sdp_mem_shape_dim(uvw, 0) != num_vis)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("The number of rows in uvw and vis must match.");
        return;
    }
    if (sdp_mem_shape_dim(uvw, 1) != 3)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("uvw must be N x 3.");
        return;
    }
    if (sdp_mem_shape_dim(freq_hz, 0) != num_chan)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("The number of channels in vis and freq_hz must match.");
        return;
    }
    if (sdp_mem_shape_dim(weight, 0) != num_vis ||
            sdp_mem_shape_dim(weight, 1) != num_chan)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("weight and vis must be the same size.");
        return;
    }
    if (have_image &&
            sdp_mem_shape_dim(dirty_image, 0) != sdp_mem_shape_dim(dirty_image, 1))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Dirty image must be square.");
        return;
    }
    const bool dbl = sdp_mem_type(uvw) == SDP_MEM_DOUBLE;
    const sdp_MemType want_real = dbl ? SDP_MEM_DOUBLE : SDP_MEM_FLOAT;
    const sdp_MemType want_cplx =
            dbl ? SDP_MEM_COMPLEX_DOUBLE : SDP_MEM_COMPLEX_FLOAT;
    if (sdp_mem_type(freq_hz) != want_real || sdp_mem_type(vis) != want_cplx ||
            sdp_mem_type(weight) != want_real ||
            sdp_mem_type(dirty_image) != want_real)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("All buffers must be the same precision.");
        return;
    }
    if (!sdp_mem_is_c_contiguous(uvw) || !sdp_mem_is_c_contiguous(freq_hz) ||
            !sdp_mem_is_c_contiguous(vis) || !sdp_mem_is_c_contiguous(weight) ||
            !sdp_mem_is_c_contiguous(dirty_image))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("All input arrays must be C contiguous");
        return;
    }
    if (do_degridding && sdp_mem_is_read_only(vis))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Visibility data must be writable.");
        return;
    }
    if (have_image && !do_degridding && sdp_mem_is_read_only(dirty_image))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Dirty image must be writable.");
        return;
    }
}

void check_parameters(double px, double py, sdp_Error* status)
{
    if (*status) return;
    if (px != py)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Only square images supported, so pixsize_x_rad and "
                "pixsize_y_rad must be equal.");
        SDP_LOG_ERROR("pixsize_x_rad is %.12e", px);
        SDP_LOG_ERROR("pixsize_y_rad is %.12e", py);
    }
}

size_t real_size(const sdp_GridderUvwEsFft* plan)
{
    return plan->is_double ? sizeof(double) : sizeof(float);
}

// Visibilities bucketed together (one batch). A call with more is split
// into row batches whose tiles are added to the grid (gridding) or whose
// visibilities are gathered from one transformed grid (degridding), so:
//  * record indices stay 32-bit: a batch lists at most 4 entries per
//    visibility (support <= 64 < tile), all below 2^32;
//  * the two worst-case record arrays stay within SDP_ES_SCRATCH_GB
//    (default 32 GiB) whatever the call size;
//  * sdp_gridder_uvw_es_fft_set_max_batch lowers the cap (tests).
int64_t batch_vis_limit(const sdp_GridderUvwEsFft* plan)
{
    static double scratch_gb = -1.0;
    if (scratch_gb < 0.0)
    {
        const char* e = getenv("SDP_ES_SCRATCH_GB");
        scratch_gb = e ? std::max(0.25, atof(e)) : 32.0;
    }
    const int64_t by_index = ((int64_t)1 << 30) - ((int64_t)1 << 20);
    const double rec_bytes = (plan->do_wstacking ? 8.0 : 4.0) *
            (plan->is_double ? 8.0 : 4.0);
    const int64_t by_mem = (int64_t)(scratch_gb * 1073741824.0 /
            (2.0 * 4.0 * rec_bytes));
    int64_t lim = std::min(by_index, by_mem);
    if (plan->max_batch_vis > 0) lim = std::min(lim, plan->max_batch_vis);
    return std::max<int64_t>(1, lim);
}

// Rows per batch for num_chan channels (a row's channels stay together).
int64_t rows_per_batch(const sdp_GridderUvwEsFft* plan, int num_chan,
        sdp_Error* status)
{
    if (*status) return 1;
    const int64_t lim = batch_vis_limit(plan);
    if (num_chan > lim)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("%d channels exceed the %lld visibilities of one "
                "bucketing batch", num_chan, (long long)lim);
        return 1;
    }
    return std::max<int64_t>(1, lim / std::max(1, num_chan));
}

// (Re)allocate the bucketing count table for num_vis visibilities.
void ensure_scratch(sdp_GridderUvwEsFft* plan, int64_t num_vis,
        sdp_Error* status)
{
    if (*status) return;
    sdp_es::BucketScratch& s = plan->scratch;
    // Worst case, so that bucketing needs no host round trip: a visibility
    // is listed in at most 4 tiles (support <= 64 < tile), work items are
    // one per bin plus one per kPiece entries.
    const size_t max_entries = 4 * (size_t)num_vis;
    const size_t items = (size_t)plan->nbins + 1 +
            (max_entries + sdp_es::kPiece - 1) / sdp_es::kPiece;
    if (items > s.item_capacity)
    {
        if (s.item_bin) SDP_HIP_CHECK(hipFree(s.item_bin), status);
        s.item_bin = nullptr;
        SDP_HIP_CHECK(hipMalloc(&s.item_bin, items * sizeof(uint32_t)),
                status);
        s.item_capacity = *status ? 0 : (uint32_t)items;
    }
    const size_t words = plan->do_wstacking ? 8 : 4;
    const size_t rec_bytes = max_entries * words * real_size(plan);
    if (rec_bytes > s.recs_bytes)
    {
        if (s.recs) SDP_HIP_CHECK(hipFree(s.recs), status);
        s.recs = nullptr;
        if (s.recs1) SDP_HIP_CHECK(hipFree(s.recs1), status);
        s.recs1 = nullptr;
        SDP_HIP_CHECK(hipMalloc(&s.recs, rec_bytes), status);
        SDP_HIP_CHECK(hipMalloc(&s.recs1, rec_bytes), status);
        s.recs_bytes = *status ? 0 : rec_bytes;
    }
    const size_t need = sdp_es::bucket_table_entries(
            sdp_es::num_chunks(num_vis, plan->tstride), plan->nbins,
            plan->nsbins);
    if (need > s.table_entries)
    {
        if (s.table) SDP_HIP_CHECK(hipFree(s.table), status);
        s.table = nullptr;
        SDP_HIP_CHECK(hipMalloc(&s.table, need * sizeof(uint32_t)), status);
        s.table_entries = *status ? 0 : need;
        s.gtable_dirty = true;
    }
}

void timing_mark(sdp_GridderUvwEsFft* plan, int k)
{
    if (plan->timing) (void)hipEventRecord(plan->ev[k], plan->stream);
}

// Sum phase times into acc_ms (syncs event k1): interval k (event k ->
// k + 1, k0 <= k < k1) is accumulated into slot[k]; slots are 0 bucketing,
// 1 scatter/gather kernel, 2 FFT, 3 image-plane kernels.
void timing_collect_range(sdp_GridderUvwEsFft* plan, int k0, int k1,
        const int slot[4])
{
    if (!plan->timing) return;
    (void)hipEventSynchronize(plan->ev[k1]);
    for (int k = k0; k < k1; ++k)
    {
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, plan->ev[k], plan->ev[k + 1]);
        plan->acc_ms[slot[k]] += ms;
    }
}

const int kGridSlots[4] = {0, 1, 2, 3};     // bucket, scatter, fft, screen
const int kDegridSlots[4] = {0, 3, 2, 1};   // bucket, screen, fft, gather

template<typename T>
sdp_es::EsParams<T> es_params(const sdp_GridderUvwEsFft* plan, int plane)
{
    sdp_es::EsParams<T> p;
    p.G = plan->grid_size;
    p.support = plan->support;
    p.do_w = plan->do_wstacking;
    p.plane = plane;
    p.ntiles = plan->ntiles;
    p.ncoarse = plan->ncoarse;
    p.ncbins = plan->ncbins;
    p.nbins = plan->nbins;
    p.sshift = plan->sshift;
    p.nsuper = plan->nsuper;
    p.nsbins = plan->nsbins;
    p.tstride = plan->tstride;
    p.beta = (T)plan->beta;
    p.uv_scale = (T)plan->uv_scale;
    p.w_scale = (T)plan->w_scale;
    p.min_plane_w = (T)plan->min_plane_w;
    memcpy(p.tap_poly, plan->tap_poly, sizeof(p.tap_poly));
    p.tap_poly_ok = plan->tap_poly_ok;
    return p;
}

template<typename T>
sdp_es::ImageParams<T> image_params(const sdp_GridderUvwEsFft* plan)
{
    sdp_es::ImageParams<T> ip;
    ip.N = plan->image_size;
    ip.G = plan->grid_size;
    ip.support = plan->support;
    ip.do_w = plan->do_wstacking;
    ip.pixel_size = (T)plan->pixel_size;
    ip.norm = (T)plan->conv_corr_norm_factor;
    ip.inv_w_scale = (T)plan->inv_w_scale;
    ip.min_plane_w = (T)plan->min_plane_w;
    const T* t = (const T*)plan->tables;
    ip.conv_corr = t;
    ip.quad_kernel = t + plan->image_size / 2 + 1;
    ip.quad_nodes = ip.quad_kernel + sdp_es::kQuadratureBound;
    ip.quad_weights = ip.quad_nodes + sdp_es::kQuadratureBound;
    return ip;
}

// Bucket + scatter one plane of this call's visibilities into grid.
template<typename T>
void scatter_plane(sdp_GridderUvwEsFft* plan, int plane, int64_t rows,
        int chan, const T* uvw, const T* freq, const T* vis, const T* weight,
        T* grid, bool skip_empty, bool accumulate, sdp_Error* status)
{
    if (*status) return;
    const sdp_es::EsParams<T> p = es_params<T>(plan, plane);
    uint32_t n_entries = 0, n_items = 0;
    timing_mark(plan, 0);
    int e = sdp_es::bucket<T>(p, sdp_es::MODE_GRID, rows, chan, uvw, freq,
            vis, weight, &plan->scratch, plan->stream, &n_entries, &n_items);
    if (e) { *status = (sdp_Error)e; return; }
    timing_mark(plan, 1);
    e = sdp_es::scatter<T>(p, plan->scratch, n_items, grid, plan->stream,
            skip_empty, accumulate);
    if (e) { *status = (sdp_Error)e; return; }
    timing_mark(plan, 2);
}

// FFT of the gridded plane + image-plane step into dirty (per plane): the
// fused pruned passes (f32, es_fft.h) or rocFFT + screen kernels.
// sparse: the grid holds only the tiles of this plane's bucketing (the
// scatter ran with skip_empty), the rest is implied zero.
template<typename T>
void grid_to_image(sdp_GridderUvwEsFft* plan,
        const sdp_es::ImageParams<T>& ip, int plane, T* grid, T* dirty,
        bool sparse, sdp_Error* status)
{
    if (*status) return;
    int e = 0;
    if constexpr (std::is_same<T, float>::value)
    {
        if (plan->fused_fft)
        {
            e = sdp_es::fft_grid_rows_cols(ip, plan->fft_tw, grid,
                    sparse ? plan->scratch.bin_count : nullptr,
                    plan->ncoarse, plan->stream);
            if (e) { *status = (sdp_Error)e; return; }
            timing_mark(plan, 3);
            e = sdp_es::fft_grid_to_image(ip, plane, plan->fft_tw, grid,
                    dirty, plan->stream);
            if (e) *status = (sdp_Error)e;
            return;
        }
    }
    sdp_fft::exec_2d(plan->fft, grid, false, plan->stream, status);
    timing_mark(plan, 3);
    if (*status) return;
    e = plan->do_wstacking ?
            sdp_es::screen_accumulate<T>(ip, plane, grid, dirty,
                    plan->stream) :
            sdp_es::screen_corr_2d<T>(ip, grid, dirty, plan->stream);
    if (e) *status = (sdp_Error)e;
}

// Gridding of rows [0, rows) in batches of rb rows into grid (zeroed
// first): every batch's tiles are added (the FFT then reads the whole grid).
// A batched 3-D call re-buckets every batch for every w-plane (planes x
// batches bucketings instead of batches): a batch's records would have to
// outlive the plane loop, and the plane's grid must hold every batch before
// its FFT, so keeping them would need one record array per batch (the
// scratch the batch limit bounds) or one grid per plane. Bucketing is ~25 %
// of a 2-D call and less of a 3-D plane; only calls past the batch limit
// (> 2^28 visibilities by default) pay it.
template<typename T>
void scatter_batches(sdp_GridderUvwEsFft* plan, int plane, int64_t rows,
        int64_t rb, int chan, const T* uvw, const T* freq, const T* vis,
        const T* weight, T* grid, sdp_Error* status)
{
    if (*status) return;
    const size_t G = (size_t)plan->grid_size;
    SDP_HIP_CHECK(hipMemsetAsync(grid, 0, G * G * 2 * real_size(plan),
            plan->stream), status);
    for (int64_t r0 = 0; r0 < rows && !*status; r0 += rb)
    {
        const int64_t n = std::min(rb, rows - r0);
        scatter_plane<T>(plan, plane, n, chan, uvw + 3 * r0, freq,
                vis + 2 * r0 * chan, weight + r0 * chan, grid, false, true,
                status);
        timing_collect_range(plan, 0, 2, kGridSlots);
    }
    timing_mark(plan, 2);
}

// Degridding: image (2-D: corrected in place) -> this plane's grid; tiles:
// the bucketing's bin counts (only the tiles the gather reads are written)
// or nullptr (every cell).
template<typename T>
void image_to_grid(sdp_GridderUvwEsFft* plan,
        const sdp_es::ImageParams<T>& ip, int plane, T* dirty, T* grid,
        const uint32_t* tiles, sdp_Error* status)
{
    if (*status) return;
    int e = 0;
    if constexpr (std::is_same<T, float>::value)
    {
        if (plan->fused_fft)
        {
            const bool in_place = !plan->do_wstacking;
            const bool real_form = sdp_es::fft_degrid_real_form(ip, in_place);
            e = sdp_es::fft_image_cols(ip, plane, plan->fft_tw, dirty,
                    in_place, real_form, grid, plan->stream);
            if (e) { *status = (sdp_Error)e; return; }
            timing_mark(plan, 2);
            // Only the tiles this plane's gather reads are written.
            e = sdp_es::fft_image_to_grid(ip, plan->fft_tw, grid, tiles,
                    plan->ncoarse, real_form, plan->stream);
            if (e) *status = (sdp_Error)e;
            return;
        }
    }
    e = sdp_es::reverse_screen<T>(ip, plane, dirty, !plan->do_wstacking,
            grid, plan->stream);
    if (e) { *status = (sdp_Error)e; return; }
    timing_mark(plan, 2);
    sdp_fft::exec_2d(plan->fft, grid, true, plan->stream, status);
}

template<typename T>
void run_grid(sdp_GridderUvwEsFft* plan, int64_t rows, int chan,
        const T* uvw, const T* freq, const T* vis, const T* weight, T* dirty,
        sdp_Error* status)
{
    const int64_t rb = rows_per_batch(plan, chan, status);
    const bool batched = rows > rb;
    ensure_scratch(plan, std::min(rows, rb) * chan, status);
    if (*status) return;
    const sdp_es::ImageParams<T> ip = image_params<T>(plan);
    T* grid = (T*)plan->grid;
    // With the fused f32 FFT the empty tiles are neither written nor read
    // (the row pass takes them from the bin counts as zeros); a batched
    // call adds every batch to a zeroed grid instead.
    const bool sparse = !batched && std::is_same<T, float>::value &&
            plan->fused_fft;
    uint32_t n_items = 0;
    if (!batched)
    {
        // One bucketing for the call: 3-D records carry their plane
        // coordinate and serve every w-plane (es_kernels.h, bucket).
        uint32_t n_entries = 0;
        timing_mark(plan, 0);
        const int e = sdp_es::bucket<T>(es_params<T>(plan, 0),
                sdp_es::MODE_GRID, rows, chan, uvw, freq, vis, weight,
                &plan->scratch, plan->stream, &n_entries, &n_items);
        if (e) { *status = (sdp_Error)e; return; }
        timing_mark(plan, 1);
        timing_collect_range(plan, 0, 1, kGridSlots);
    }
    const int nplanes = plan->num_total_w_grids;
    // Planes per 3-D tile-kernel pass: the extra planes' grids are allocated
    // on first use (G^2 complex each: 2 GiB at G = 16384). An allocation
    // that fails is not an error: the pass takes the planes that have a
    // grid, down to the single-plane path the call ran before.
    auto pass_planes = [&](int plane) -> int {
        if (batched || plane + 1 >= nplanes) return 1;
        int np = std::min(nplanes - plane,
                sdp_es::planes_per_pass(es_params<T>(plan, plane)));
        const size_t cells = (size_t)plan->grid_size * plan->grid_size;
        for (int q = 1; q < np; ++q)
        {
            if (plan->grid_x[q - 1]) continue;
            if (hipMalloc(&plan->grid_x[q - 1], cells * 2 * sizeof(T)) !=
                    hipSuccess)
            {
                plan->grid_x[q - 1] = nullptr;
                (void)hipGetLastError();   // clear the sticky error
                SDP_LOG_WARNING("3-D gridding: no memory for a second "
                        "w-plane grid; one plane per tile-kernel pass");
                return q;
            }
        }
        return np;
    };
    for (int plane = 0; plane < nplanes && !*status; ++plane)
    {
        const int np = pass_planes(plane);
        if (batched)
        {
            scatter_batches<T>(plan, plane, rows, rb, chan, uvw, freq, vis,
                    weight, grid, status);
        }
        else if (np > 1)
        {
            // 3-D: this plane and the next one or two in one tile-kernel
            // pass (the entries' staging is shared), the others into
            // plan-owned grids; then each plane's FFT and image step.
            T* grids[3] = {grid, nullptr, nullptr};
            for (int q = 1; q < np; ++q) grids[q] = (T*)plan->grid_x[q - 1];
            timing_mark(plan, 1);
            int e = sdp_es::scatter_planes<T>(es_params<T>(plan, plane),
                    plan->scratch, n_items, grids, np, plan->stream, sparse);
            if (e) { *status = (sdp_Error)e; return; }
            for (int q = 0; q < np; ++q, ++plane)
            {
                timing_mark(plan, 2);
                grid_to_image<T>(plan, ip, plane, grids[q], dirty, sparse,
                        status);
                if (*status) return;
                if (plane == nplanes - 1)
                {
                    e = sdp_es::apply_correction<T>(ip, dirty, plan->stream);
                    if (e) { *status = (sdp_Error)e; return; }
                }
                timing_mark(plan, 4);
                timing_collect_range(plan, q == 0 ? 1 : 2, 4, kGridSlots);
            }
            --plane;            // the loop's ++plane moves past the last
            continue;
        }
        else
        {
            timing_mark(plan, 1);
            const int e = sdp_es::scatter<T>(es_params<T>(plan, plane),
                    plan->scratch, n_items, grid, plan->stream, sparse,
                    false);
            if (e) { *status = (sdp_Error)e; return; }
            timing_mark(plan, 2);
        }
        grid_to_image<T>(plan, ip, plane, grid, dirty, sparse, status);
        if (*status) return;
        if (plan->do_wstacking && plane == plan->num_total_w_grids - 1)
        {
            const int e = sdp_es::apply_correction<T>(ip, dirty, plan->stream);
            if (e) { *status = (sdp_Error)e; return; }
        }
        timing_mark(plan, 4);
        timing_collect_range(plan, batched ? 2 : 1, 4, kGridSlots);
    }
}

// Degridding of one plane in batches of rb rows: the image side writes
// every grid cell once, then each batch is bucketed and gathered.
template<typename T>
void degrid_batches(sdp_GridderUvwEsFft* plan,
        const sdp_es::ImageParams<T>& ip, int plane, int64_t rows,
        int64_t rb, int chan, const T* uvw, const T* freq, T* vis, T* dirty,
        sdp_Error* status)
{
    if (*status) return;
    T* grid = (T*)plan->grid;
    timing_mark(plan, 1);
    image_to_grid<T>(plan, ip, plane, dirty, grid, nullptr, status);
    if (*status) return;
    timing_mark(plan, 3);
    timing_collect_range(plan, 1, 3, kDegridSlots);
    for (int64_t r0 = 0; r0 < rows; r0 += rb)
    {
        const int64_t n = std::min(rb, rows - r0);
        const sdp_es::EsParams<T> p = es_params<T>(plan, plane);
        uint32_t n_entries = 0, n_items = 0;
        timing_mark(plan, 0);
        int e = sdp_es::bucket<T>(p, sdp_es::MODE_DEGRID, n, chan,
                uvw + 3 * r0, freq, nullptr, nullptr, &plan->scratch,
                plan->stream, &n_entries, &n_items);
        if (e) { *status = (sdp_Error)e; return; }
        timing_mark(plan, 1);
        e = sdp_es::gather<T>(p, plan->scratch, n_items, grid,
                vis + 2 * r0 * chan, plan->stream);
        if (e) { *status = (sdp_Error)e; return; }
        timing_mark(plan, 2);
        const int slots[4] = {0, 1, 0, 0};
        timing_collect_range(plan, 0, 2, slots);
    }
}

template<typename T>
void run_degrid(sdp_GridderUvwEsFft* plan, int64_t rows, int chan,
        const T* uvw, const T* freq, T* vis, T* dirty, sdp_Error* status)
{
    const int64_t rb = rows_per_batch(plan, chan, status);
    const bool batched = rows > rb;
    ensure_scratch(plan, std::min(rows, rb) * chan, status);
    if (*status) return;
    const sdp_es::ImageParams<T> ip = image_params<T>(plan);
    T* grid = (T*)plan->grid;
    int e = 0;
    if (plan->do_wstacking)
    {
        e = sdp_es::apply_correction<T>(ip, dirty, plan->stream);
        if (e) { *status = (sdp_Error)e; return; }
    }
    uint32_t n_items = 0;
    if (!batched)
    {
        // One bucketing for the call (3-D: for every w-plane).
        uint32_t n_entries = 0;
        timing_mark(plan, 0);
        e = sdp_es::bucket<T>(es_params<T>(plan, 0), sdp_es::MODE_DEGRID,
                rows, chan, uvw, freq, nullptr, nullptr, &plan->scratch,
                plan->stream, &n_entries, &n_items);
        if (e) { *status = (sdp_Error)e; return; }
        timing_mark(plan, 1);
        timing_collect_range(plan, 0, 1, kDegridSlots);
    }
    for (int plane = 0; plane < plan->num_total_w_grids && !*status; ++plane)
    {
        if (batched)
        {
            degrid_batches<T>(plan, ip, plane, rows, rb, chan, uvw, freq,
                    vis, dirty, status);
            continue;
        }
        timing_mark(plan, 1);
        image_to_grid<T>(plan, ip, plane, dirty, grid,
                plan->scratch.bin_count, status);
        if (*status) return;
        timing_mark(plan, 3);
        e = sdp_es::gather<T>(es_params<T>(plan, plane), plan->scratch,
                n_items, grid, vis, plan->stream);
        if (e) { *status = (sdp_Error)e; return; }
        timing_mark(plan, 4);
        timing_collect_range(plan, 1, 4, kDegridSlots);
    }
}

void timing_begin(sdp_GridderUvwEsFft* plan)
{
    for (int k = 0; k < 5; ++k) plan->acc_ms[k] = 0.0;
    plan->have_timing = 0;
}

void timing_end(sdp_GridderUvwEsFft* plan, double wall_ms)
{
    if (!plan->timing) return;
    plan->acc_ms[4] = wall_ms;
    plan->have_timing = 1;
}

// Grid (and image) arguments of the row-spectra halves: a fused-FFT 2-D
// f32 plan and its G x G complex grid on the GPU.
float* row_split_grid(sdp_GridderUvwEsFft* plan, sdp_Mem* grid,
        sdp_Error* status)
{
    if (*status || !plan) return nullptr;
    if (!sdp_gridder_uvw_es_fft_row_spectra(plan, nullptr, nullptr, nullptr))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Row-spectra split needs a 2-D single-precision plan "
                "with a power-of-two grid");
        return nullptr;
    }
    const int64_t G = plan->grid_size;
    if (sdp_mem_type(grid) != SDP_MEM_COMPLEX_FLOAT ||
            sdp_mem_num_dims(grid) != 2 || sdp_mem_shape_dim(grid, 0) != G ||
            sdp_mem_shape_dim(grid, 1) != G || !sdp_mem_is_c_contiguous(grid))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("grid must be a contiguous %lld x %lld complex float "
                "array", (long long)G, (long long)G);
        return nullptr;
    }
    void* p = sdp_mem_gpu_buffer(grid, status);
    return *status ? nullptr : *(float**)p;
}


} // namespace

extern "C" {

void sdp_gridder_uvw_es_fft_free_plan(sdp_GridderUvwEsFft* plan)
{
    if (!plan) return;
    if (plan->grid) (void)hipFree(plan->grid);
    for (void* g : plan->grid_x)
        if (g) (void)hipFree(g);
    if (plan->tables) (void)hipFree(plan->tables);
    sdp_es::BucketScratch& s = plan->scratch;
    if (s.table) (void)hipFree(s.table);
    if (s.item_bin) (void)hipFree(s.item_bin);
    if (s.bin_count) (void)hipFree(s.bin_count);
    if (s.recs) (void)hipFree(s.recs);
    if (s.recs1) (void)hipFree(s.recs1);
    sdp_fft::destroy_2d(plan->fft);
    sdp_es::fft_twiddles_destroy(&plan->fft_tw);
    if (plan->timing)
        for (int k = 0; k < 5; ++k) (void)hipEventDestroy(plan->ev[k]);
    free(plan);
}

sdp_GridderUvwEsFft* sdp_gridder_uvw_es_fft_create_plan(
        const sdp_Mem* uvw, const sdp_Mem* freq_hz, const sdp_Mem* vis,
        const sdp_Mem* weight, const sdp_Mem* dirty_image,
        const double pixel_size_x_rad, const double pixel_size_y_rad,
        const double epsilon, const double min_abs_w, const double max_abs_w,
        const int do_w_stacking, sdp_Error* status)
{
    if (*status) return nullptr;
    check_parameters(pixel_size_x_rad, pixel_size_y_rad, status);
    check_buffers(uvw, freq_hz, vis, weight, dirty_image, false, status);
    if (*status) return nullptr;

    sdp_GridderUvwEsFft* plan =
            (sdp_GridderUvwEsFft*)calloc(1, sizeof(sdp_GridderUvwEsFft));
    plan->pixsize_x_rad = pixel_size_x_rad;
    plan->pixsize_y_rad = pixel_size_y_rad;
    plan->pixel_size = pixel_size_x_rad;
    plan->epsilon = epsilon;
    plan->do_wstacking = do_w_stacking ? 1 : 0;
    plan->num_rows = (int)sdp_mem_shape_dim(vis, 0);
    plan->num_chan = (int)sdp_mem_shape_dim(vis, 1);
    plan->image_size = (int)sdp_mem_shape_dim(dirty_image, 0);
    plan->is_double = (sdp_mem_type(vis) & SDP_MEM_DOUBLE) ? 1 : 0;

    double beta_w = 0.0;
    sdp_es::params_from_epsilon(epsilon, plan->image_size,
            plan->is_double != 0, &plan->grid_size, &plan->support, &beta_w);
    plan->beta = beta_w * plan->support;
    plan->uv_scale = plan->grid_size * plan->pixel_size;
    // Interior taps as polynomials (f32 tile kernels, W = 8), fitted to the
    // beta the f32 kernels use.
    if (!plan->is_double && plan->support == 8)
    {
        sdp_es::es_tap_poly_fit((double)(float)plan->beta, plan->tap_poly);
        plan->tap_poly_ok = 1;
    }

    // w-plane geometry, sdp_gridder_uvw_es_fft.cpp:346-383.
    if (plan->do_wstacking)
    {
        const double x0 = -0.5 * plan->image_size * plan->pixel_size;
        const double y0 = x0;
        double nmin = sqrt(std::max(1.0 - x0 * x0 - y0 * y0, 0.0)) - 1.0;
        if (x0 * x0 + y0 * y0 > 1.0)
        {
            nmin = -sqrt(fabs(1.0 - x0 * x0 - y0 * y0)) - 1.0;
        }
        double w_scale = 0.25 / fabs(nmin);
        int nw = (int)((max_abs_w - min_abs_w) / w_scale + 2);
        w_scale = 1.0 / ((1.0 + 1e-13) * (max_abs_w - min_abs_w) / (nw - 1));
        plan->min_plane_w = min_abs_w - (0.5 * plan->support - 1.0) / w_scale;
        plan->max_plane_w = max_abs_w + (0.5 * plan->support - 1.0) / w_scale;
        plan->num_total_w_grids = nw + plan->support - 2;
        plan->min_abs_w = min_abs_w;
        plan->max_abs_w = max_abs_w;
        plan->w_scale = w_scale;
        plan->inv_w_range = plan->max_plane_w - plan->min_plane_w;
    }
    else
    {
        plan->num_total_w_grids = 1;
        plan->inv_w_range = 1.0;
        plan->w_scale = 1.0;
    }
    plan->inv_w_scale = 1.0 / plan->w_scale;

    // Correction tables (host, double), then cast to working precision.
    const int nc = plan->image_size / 2 + 1;
    const int q = sdp_es::kQuadratureBound;
    double* host = (double*)calloc(nc + 3 * q, sizeof(double));
    plan->conv_corr_norm_factor = sdp_es::gauss_legendre_conv_kernel(
            plan->image_size, plan->grid_size, plan->support, plan->beta,
            host + nc, host + nc + q, host + nc + 2 * q, host);
    plan->ntiles = (plan->grid_size + sdp_es::kTile - 1) / sdp_es::kTile;
    plan->ncoarse = (plan->grid_size + sdp_es::kCoarseTile - 1) /
            sdp_es::kCoarseTile;
    plan->ncbins = plan->ncoarse * plan->ncoarse;
    plan->nbins = plan->ncbins * sdp_es::kCoarse * sdp_es::kCoarse;
    plan->stream = 0;
    if (!sdp_es::super_geometry(plan->ntiles, &plan->sshift, &plan->nsuper,
            &plan->nsbins))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Grid size %d too large for the bucketing",
                plan->grid_size);
        free(host);
        sdp_gridder_uvw_es_fft_free_plan(plan);
        return nullptr;
    }
    plan->tstride = plan->nbins + plan->nsbins;

    if (!sdp_hip::device_available())
    {
        // Same outcome as the reference built without GPU support.
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Cannot allocate GPU memory: no HIP device available.");
        free(host);
        sdp_gridder_uvw_es_fft_free_plan(plan);
        return nullptr;
    }
    const size_t rs = real_size(plan);
    const size_t ntab = nc + 3 * q;
    SDP_HIP_CHECK(hipMalloc(&plan->tables, ntab * rs), status);
    if (!*status)
    {
        if (plan->is_double)
        {
            SDP_HIP_CHECK(hipMemcpy(plan->tables, host, ntab * rs,
                    hipMemcpyHostToDevice), status);
        }
        else
        {
            float* f = (float*)malloc(ntab * sizeof(float));
            for (size_t i = 0; i < ntab; ++i) f[i] = (float)host[i];
            SDP_HIP_CHECK(hipMemcpy(plan->tables, f, ntab * rs,
                    hipMemcpyHostToDevice), status);
            free(f);
        }
    }
    free(host);
    const size_t cells = (size_t)plan->grid_size * plan->grid_size;
    SDP_HIP_CHECK(hipMalloc(&plan->grid, cells * 2 * rs), status);
    sdp_es::BucketScratch& s = plan->scratch;
    const size_t nb = (size_t)plan->nbins;
    if (!*status)
    {
        // bin_count (tile then super-bin totals) | bin_start | item_start |
        // totals in one allocation.
        SDP_HIP_CHECK(hipMalloc(&s.bin_count,
                (plan->tstride + 2 * (nb + 1) + 2 + plan->nsbins + 1) *
                sizeof(uint32_t)), status);
        if (!*status)
        {
            s.bin_start = s.bin_count + plan->tstride;
            s.item_start = s.bin_start + nb + 1;
            s.totals = s.item_start + nb + 1;
            s.sb_start = s.totals + 2;
        }
    }
    ensure_scratch(plan, std::min((int64_t)plan->num_rows * plan->num_chan,
            batch_vis_limit(plan)), status);
    // SDP_ES_FFT=rocfft keeps rocFFT + separate screen kernels for f32 too.
    const char* fft_env = getenv("SDP_ES_FFT");
    plan->fused_fft = !plan->is_double &&
            sdp_es::fused_fft_supported(plan->grid_size) &&
            !(fft_env && strcmp(fft_env, "rocfft") == 0);
    if (plan->fused_fft)
    {
        const int e = sdp_es::fft_twiddles_create(plan->grid_size,
                &plan->fft_tw);
        if (e && !*status) *status = (sdp_Error)e;
    }
    else
    {
        plan->fft = sdp_fft::create_2d(plan->grid_size, plan->grid_size,
                plan->is_double != 0, status);
    }
    if (*status)
    {
        if (*status == SDP_ERR_RUNTIME) *status = SDP_ERR_MEM_ALLOC_FAILURE;
        sdp_gridder_uvw_es_fft_free_plan(plan);
        return nullptr;
    }
    return plan;
}

void sdp_grid_uvw_es_fft(sdp_GridderUvwEsFft* plan, const sdp_Mem* uvw,
        const sdp_Mem* freq_hz, const sdp_Mem* vis, const sdp_Mem* weight,
        sdp_Mem* dirty_image, sdp_Error* status)
{
    SDP_LOG_DEBUG("Executing sdp_GridderUvwEsFft...");
    if (*status || !plan) return;
    check_parameters(plan->pixsize_x_rad, plan->pixsize_y_rad, status);
    check_buffers(uvw, freq_hz, vis, weight, dirty_image, false, status);
    if (*status) return;
    // Device pointers (fails with SDP_ERR_MEM_LOCATION for host memory).
    const void* p_uvw = sdp_mem_gpu_buffer_const(uvw, status);
    const void* p_freq = sdp_mem_gpu_buffer_const(freq_hz, status);
    const void* p_vis = sdp_mem_gpu_buffer_const(vis, status);
    const void* p_wt = sdp_mem_gpu_buffer_const(weight, status);
    void* p_dirty = sdp_mem_gpu_buffer(dirty_image, status);
    if (*status) return;
    if (sdp_mem_shape_dim(dirty_image, 0) != plan->image_size ||
            (int)sdp_mem_is_double(vis) != plan->is_double)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Buffers do not match those used to create the plan");
        return;
    }
    const int64_t rows = sdp_mem_shape_dim(vis, 0);
    const int chan = (int)sdp_mem_shape_dim(vis, 1);
    timing_begin(plan);
    if (plan->is_double)
        run_grid<double>(plan, rows, chan, *(const double* const*)p_uvw,
                *(const double* const*)p_freq, *(const double* const*)p_vis,
                *(const double* const*)p_wt, *(double**)p_dirty, status);
    else
        run_grid<float>(plan, rows, chan, *(const float* const*)p_uvw,
                *(const float* const*)p_freq, *(const float* const*)p_vis,
                *(const float* const*)p_wt, *(float**)p_dirty, status);
    timing_end(plan, 0.0);
}

void sdp_ifft_degrid_uvw_es(sdp_GridderUvwEsFft* plan, const sdp_Mem* uvw,
        const sdp_Mem* freq_hz, sdp_Mem* vis, const sdp_Mem* weight,
        sdp_Mem* dirty_image, sdp_Error* status)
{
    SDP_LOG_DEBUG("Executing sdp_GridderUvwEsFft...");
    if (*status || !plan) return;
    check_parameters(plan->pixsize_x_rad, plan->pixsize_y_rad, status);
    check_buffers(uvw, freq_hz, vis, weight, dirty_image, true, status);
    if (*status) return;
    const void* p_uvw = sdp_mem_gpu_buffer_const(uvw, status);
    const void* p_freq = sdp_mem_gpu_buffer_const(freq_hz, status);
    void* p_vis = sdp_mem_gpu_buffer(vis, status);
    (void)sdp_mem_gpu_buffer_const(weight, status);
    void* p_dirty = sdp_mem_gpu_buffer(dirty_image, status);
    if (*status) return;
    if (sdp_mem_shape_dim(dirty_image, 0) != plan->image_size ||
            (int)sdp_mem_is_double(vis) != plan->is_double)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Buffers do not match those used to create the plan");
        return;
    }
    const int64_t rows = sdp_mem_shape_dim(vis, 0);
    const int chan = (int)sdp_mem_shape_dim(vis, 1);
    timing_begin(plan);
    if (plan->is_double)
        run_degrid<double>(plan, rows, chan, *(const double* const*)p_uvw,
                *(const double* const*)p_freq, *(double**)p_vis,
                *(double**)p_dirty, status);
    else
        run_degrid<float>(plan, rows, chan, *(const float* const*)p_uvw,
                *(const float* const*)p_freq, *(float**)p_vis,
                *(float**)p_dirty, status);
    timing_end(plan, 0.0);
}

void sdp_gridder_uvw_es_fft_params_from_epsilon(double epsilon,
        int image_size, int is_double, int* grid_size, int* support,
        double* beta_over_support)
{
    sdp_es::params_from_epsilon(epsilon, image_size, is_double != 0,
            grid_size, support, beta_over_support);
}

int sdp_gridder_uvw_es_fft_grid_size(const sdp_GridderUvwEsFft* plan)
{
    return plan ? plan->grid_size : 0;
}

int sdp_gridder_uvw_es_fft_support(const sdp_GridderUvwEsFft* plan)
{
    return plan ? plan->support : 0;
}

int sdp_gridder_uvw_es_fft_num_w_planes(const sdp_GridderUvwEsFft* plan)
{
    return plan ? plan->num_total_w_grids : 0;
}

double sdp_gridder_uvw_es_fft_beta(const sdp_GridderUvwEsFft* plan)
{
    return plan ? plan->beta : 0.0;
}

int sdp_gridder_uvw_es_fft_fused_fft(const sdp_GridderUvwEsFft* plan)
{
    return plan ? plan->fused_fft : 0;
}

void sdp_gridder_uvw_es_fft_set_stream(sdp_GridderUvwEsFft* plan,
        void* hip_stream)
{
    if (!plan || plan->stream == (hipStream_t)hip_stream) return;
    // Every call reuses the plan's grid, records and count tables, and the
    // next bucketing counts into group rows that the previous call's
    // k_bucket_fill2 clears: the work queued on the old stream must finish
    // before anything is queued on the new one.
    if (hipStreamSynchronize(plan->stream) != hipSuccess)
        plan->scratch.gtable_dirty = true;
    plan->stream = (hipStream_t)hip_stream;
}

void sdp_gridder_uvw_es_fft_enable_timing(sdp_GridderUvwEsFft* plan,
        int enable)
{
    if (!plan || (enable != 0) == (plan->timing != 0)) return;
    for (int k = 0; k < 5; ++k)
    {
        if (enable) (void)hipEventCreate(&plan->ev[k]);
        else (void)hipEventDestroy(plan->ev[k]);
    }
    plan->timing = enable ? 1 : 0;
    plan->have_timing = 0;
}

int sdp_gridder_uvw_es_fft_get_timing(sdp_GridderUvwEsFft* plan,
        double* out_ms, int max_values)
{
    if (!plan || !plan->timing || !plan->have_timing) return 0;
    double total = 0.0;
    for (int k = 0; k < 4; ++k) total += plan->acc_ms[k];
    plan->acc_ms[4] = total;
    const int n = max_values < 5 ? max_values : 5;
    for (int k = 0; k < n; ++k) out_ms[k] = plan->acc_ms[k];
    return n;
}

void sdp_grid_uvw_es_fft_scatter(sdp_GridderUvwEsFft* plan,
        const sdp_Mem* uvw, const sdp_Mem* freq_hz, const sdp_Mem* vis,
        const sdp_Mem* weight, sdp_Mem* grid, sdp_Error* status)
{
    if (*status || !plan) return;
    if (plan->do_wstacking)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Split gridding is only available for 2-D plans");
        return;
    }
    // Reuse the standard checks with the grid standing in for the image.
    check_buffers(uvw, freq_hz, vis, weight, nullptr, false, status);
    if (*status) return;
    const int64_t G = plan->grid_size;
    const sdp_MemType gt = plan->is_double ? SDP_MEM_COMPLEX_DOUBLE :
            SDP_MEM_COMPLEX_FLOAT;
    if (sdp_mem_type(grid) != gt || sdp_mem_num_dims(grid) != 2 ||
            sdp_mem_shape_dim(grid, 0) != G || sdp_mem_shape_dim(grid, 1) != G ||
            !sdp_mem_is_c_contiguous(grid))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("grid must be a contiguous %lld x %lld complex array "
                "of the plan's precision", (long long)G, (long long)G);
        return;
    }
    const void* p_uvw = sdp_mem_gpu_buffer_const(uvw, status);
    const void* p_freq = sdp_mem_gpu_buffer_const(freq_hz, status);
    const void* p_vis = sdp_mem_gpu_buffer_const(vis, status);
    const void* p_wt = sdp_mem_gpu_buffer_const(weight, status);
    void* p_grid = sdp_mem_gpu_buffer(grid, status);
    if (*status) return;
    const int64_t rows = sdp_mem_shape_dim(vis, 0);
    const int chan = (int)sdp_mem_shape_dim(vis, 1);
    const int64_t rb = rows_per_batch(plan, chan, status);
    ensure_scratch(plan, std::min(rows, rb) * chan, status);
    timing_begin(plan);
#define SDP_ES_SPLIT(T) \
    if (rows > rb) \
        scatter_batches<T>(plan, 0, rows, rb, chan, *(const T* const*)p_uvw, \
                *(const T* const*)p_freq, *(const T* const*)p_vis, \
                *(const T* const*)p_wt, *(T**)p_grid, status); \
    else \
        scatter_plane<T>(plan, 0, rows, chan, *(const T* const*)p_uvw, \
                *(const T* const*)p_freq, *(const T* const*)p_vis, \
                *(const T* const*)p_wt, *(T**)p_grid, false, false, status);
    if (plan->is_double) { SDP_ES_SPLIT(double) }
    else { SDP_ES_SPLIT(float) }
#undef SDP_ES_SPLIT
}

void sdp_gridder_uvw_es_fft_set_max_batch(sdp_GridderUvwEsFft* plan,
        int64_t max_vis)
{
    if (plan) plan->max_batch_vis = max_vis > 0 ? max_vis : 0;
}

int64_t sdp_gridder_uvw_es_fft_batch_vis(const sdp_GridderUvwEsFft* plan)
{
    return plan ? batch_vis_limit(plan) : 0;
}

void sdp_grid_uvw_es_fft_finish(sdp_GridderUvwEsFft* plan, sdp_Mem* grid,
        sdp_Mem* dirty_image, sdp_Error* status)
{
    if (*status || !plan) return;
    if (plan->do_wstacking)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Split gridding is only available for 2-D plans");
        return;
    }
    const int64_t G = plan->grid_size;
    const sdp_MemType gt = plan->is_double ? SDP_MEM_COMPLEX_DOUBLE :
            SDP_MEM_COMPLEX_FLOAT;
    const sdp_MemType it = plan->is_double ? SDP_MEM_DOUBLE : SDP_MEM_FLOAT;
    if (sdp_mem_type(grid) != gt || sdp_mem_shape_dim(grid, 0) != G ||
            sdp_mem_shape_dim(grid, 1) != G || !sdp_mem_is_c_contiguous(grid) ||
            sdp_mem_type(dirty_image) != it ||
            sdp_mem_shape_dim(dirty_image, 0) != plan->image_size ||
            sdp_mem_shape_dim(dirty_image, 1) != plan->image_size ||
            !sdp_mem_is_c_contiguous(dirty_image))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("grid / dirty_image do not match the plan");
        return;
    }
    void* p_grid = sdp_mem_gpu_buffer(grid, status);
    void* p_dirty = sdp_mem_gpu_buffer(dirty_image, status);
    if (*status) return;
    if (plan->is_double)
        grid_to_image<double>(plan, image_params<double>(plan), 0,
                *(double**)p_grid, *(double**)p_dirty, false, status);
    else
        grid_to_image<float>(plan, image_params<float>(plan), 0,
                *(float**)p_grid, *(float**)p_dirty, false, status);
}

int sdp_gridder_uvw_es_fft_row_spectra(const sdp_GridderUvwEsFft* plan,
        int64_t* rows, int64_t* col0, int64_t* ncols)
{
    if (!plan || plan->is_double || !plan->fused_fft || plan->do_wstacking)
        return 0;
    int64_t r = 0, c = 0, n = 0;
    sdp_es::fft_grid_row_spectra(image_params<float>(plan), &r, &c, &n);
    if (rows) *rows = r;
    if (col0) *col0 = c;
    if (ncols) *ncols = n;
    return 1;
}


void sdp_grid_uvw_es_fft_rows(sdp_GridderUvwEsFft* plan, sdp_Mem* grid,
        sdp_Error* status)
{
    float* g = row_split_grid(plan, grid, status);
    if (*status) return;
    const int e = sdp_es::fft_grid_rows(image_params<float>(plan),
            plan->fft_tw, g, nullptr, plan->ncoarse, plan->stream);
    if (e) *status = (sdp_Error)e;
}

void sdp_grid_uvw_es_fft_finish_rows(sdp_GridderUvwEsFft* plan,
        sdp_Mem* grid, sdp_Mem* dirty_image, sdp_Error* status)
{
    float* g = row_split_grid(plan, grid, status);
    if (*status) return;
    if (sdp_mem_type(dirty_image) != SDP_MEM_FLOAT ||
            sdp_mem_num_dims(dirty_image) != 2 ||
            sdp_mem_shape_dim(dirty_image, 0) != plan->image_size ||
            sdp_mem_shape_dim(dirty_image, 1) != plan->image_size ||
            !sdp_mem_is_c_contiguous(dirty_image))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("dirty_image does not match the plan");
        return;
    }
    void* p_dirty = sdp_mem_gpu_buffer(dirty_image, status);
    if (*status) return;
    const sdp_es::ImageParams<float> ip = image_params<float>(plan);
    int e = sdp_es::fft_grid_cols_a(ip, plan->fft_tw, g, plan->stream);
    if (!e)
        e = sdp_es::fft_grid_to_image(ip, 0, plan->fft_tw, g,
                *(float**)p_dirty, plan->stream);
    if (e) *status = (sdp_Error)e;
}

} // extern "C"
