/* MI355X-native ES-FFT (de)gridder: drop-in C ABI.
 *
 * Entry points replace, symbol for symbol and argument for argument,
 *   src/ska-sdp-func/grid_data/sdp_gridder_uvw_es_fft.h:42-116
 * of ska-sdp-func 1.2.2 (bound from Python by
 *   src/ska_sdp_func/grid_data/gridder_uvw_es_fft.py:149-200).
 *
 * Semantics kept from the reference (sdp_gridder_uvw_es_fft.cpp):
 *  - every buffer must be in GPU memory, C-contiguous, of one precision; a
 *    host buffer fails with SDP_ERR_MEM_LOCATION (there is no CPU path);
 *  - u is the grid ROW (slow) axis; taps outside the grid are dropped;
 *  - gridding ACCUMULATES into dirty_image and multiplies the whole image
 *    (including what the caller had in it) by the correction;
 *  - degridding applies the correction IN PLACE on dirty_image, ignores
 *    weights and accumulates into vis;
 *  - 3-D (w-stacking): w < 0 rows are flipped and conjugated.
 * Launches are asynchronous on the plan's HIP stream (default: the null
 * stream), as the reference launches on stream 0.
 */
#ifndef SDP_GRID_UVW_ES_FFT_H_
#define SDP_GRID_UVW_ES_FFT_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

struct sdp_GridderUvwEsFft;
typedef struct sdp_GridderUvwEsFft sdp_GridderUvwEsFft;

/* sdp_gridder_uvw_es_fft.h:42-55 (impl .cpp:276-529) */
sdp_GridderUvwEsFft* sdp_gridder_uvw_es_fft_create_plan(
        const sdp_Mem* uvw,
        const sdp_Mem* freq_hz,
        const sdp_Mem* vis,
        const sdp_Mem* weight,
        const sdp_Mem* dirty_image,
        const double pixel_size_x_rad,
        const double pixel_size_y_rad,
        const double epsilon,
        const double min_abs_w,
        const double max_abs_w,
        const int do_w_stacking,
        sdp_Error* status
);

/* sdp_gridder_uvw_es_fft.h:71-79 (impl .cpp:532-742) */
void sdp_grid_uvw_es_fft(
        sdp_GridderUvwEsFft* plan,
        const sdp_Mem* uvw,
        const sdp_Mem* freq_hz,
        const sdp_Mem* vis,
        const sdp_Mem* weight,
        sdp_Mem* dirty_image,
        sdp_Error* status
);

/* sdp_gridder_uvw_es_fft.h:95-103 (impl .cpp:745-956) */
void sdp_ifft_degrid_uvw_es(
        sdp_GridderUvwEsFft* plan,
        const sdp_Mem* uvw,
        const sdp_Mem* freq_hz,
        sdp_Mem* vis,
        const sdp_Mem* weight,
        sdp_Mem* dirty_image,
        sdp_Error* status
);

/* sdp_gridder_uvw_es_fft.h:110-113 (impl .cpp:60-69) */
void sdp_gridder_uvw_es_fft_free_plan(sdp_GridderUvwEsFft* plan);

/* ---- MI355X extensions (not in the reference ABI) -------------------- */

/* Kernel parameters the plan would choose (no GPU needed): grid size,
 * support and beta/support for (epsilon, image size, precision); follows
 * sdp_calculate_params_from_epsilon (sdp_gridder_uvw_es_fft_utils.cpp:225). */
void sdp_gridder_uvw_es_fft_params_from_epsilon(double epsilon,
        int image_size, int is_double, int* grid_size, int* support,
        double* beta_over_support);

/* Plan geometry accessors. */
int sdp_gridder_uvw_es_fft_grid_size(const sdp_GridderUvwEsFft* plan);
int sdp_gridder_uvw_es_fft_support(const sdp_GridderUvwEsFft* plan);
int sdp_gridder_uvw_es_fft_num_w_planes(const sdp_GridderUvwEsFft* plan);
double sdp_gridder_uvw_es_fft_beta(const sdp_GridderUvwEsFft* plan);

/* 1 if the plan uses the pruned, fused FFT passes (f32, power-of-two grid
 * of 1024..16384 cells; environment SDP_ES_FFT=rocfft at plan creation
 * selects rocFFT + separate screen kernels instead), 0 for rocFFT. */
int sdp_gridder_uvw_es_fft_fused_fft(const sdp_GridderUvwEsFft* plan);

/* Calls are bucketed in batches of at most sdp_gridder_uvw_es_fft_batch_vis
 * visibilities (whole rows): a larger call is split into row batches that
 * are added into one grid (gridding) or gathered from one transformed grid
 * (degridding), so bucketing indices stay 32-bit and the record scratch
 * stays within SDP_ES_SCRATCH_GB (default 32 GiB). Results equal the
 * unbatched call up to summation order. set_max_batch lowers the cap
 * (0 = the default); a row with more channels than the cap is an invalid
 * argument. */
void sdp_gridder_uvw_es_fft_set_max_batch(sdp_GridderUvwEsFft* plan,
        int64_t max_vis);
int64_t sdp_gridder_uvw_es_fft_batch_vis(const sdp_GridderUvwEsFft* plan);

/* Run the plan's work on a caller-owned hipStream_t (NULL = null stream).
 * Switching to another stream first waits for the work queued on the old
 * one (the plan's grid and scratch are shared by consecutive calls). */
void sdp_gridder_uvw_es_fft_set_stream(sdp_GridderUvwEsFft* plan,
        void* hip_stream);

/* Per-phase device timing (HIP events on the plan stream) of the last
 * grid/degrid call: out_ms[0] bucketing, [1] scatter or gather kernel,
 * [2] FFT, [3] image-plane kernels, [4] whole call. Returns the number of
 * values written (0 if timing is disabled). Synchronises the events. */
void sdp_gridder_uvw_es_fft_enable_timing(sdp_GridderUvwEsFft* plan,
        int enable);
int sdp_gridder_uvw_es_fft_get_timing(sdp_GridderUvwEsFft* plan,
        double* out_ms, int max_values);

/* Split 2-D gridding for multi-GPU row sharding: scatter this process's
 * rows into a caller-owned G x G complex grid (every cell written), then,
 * after the caller has summed the per-GPU grids (e.g. RCCL reduce),
 * finish = inverse FFT (in place on grid) + screen + correction into
 * dirty_image. scatter + finish == sdp_grid_uvw_es_fft for 2-D plans. */
void sdp_grid_uvw_es_fft_scatter(
        sdp_GridderUvwEsFft* plan,
        const sdp_Mem* uvw,
        const sdp_Mem* freq_hz,
        const sdp_Mem* vis,
        const sdp_Mem* weight,
        sdp_Mem* grid,
        sdp_Error* status
);
void sdp_grid_uvw_es_fft_finish(
        sdp_GridderUvwEsFft* plan,
        sdp_Mem* grid,
        sdp_Mem* dirty_image,
        sdp_Error* status
);

/* MI355X extension: finish in two halves around a reduction of row
 * spectra (multi-GPU "grid" mode; the split of the reference's inverse
 * FFT, sdp_gridder_uvw_es_fft.cpp:660-701).
 * _rows runs the first pass of the inverse FFT (the row FFTs, real-output
 * form where the plan uses it) in place on a scattered grid; the data the
 * remaining passes read is then grid rows [0, rows) x columns [col0, col0
 * + ncols), reported by _row_spectra (returns 0 for plans without the
 * fused f32 FFT: f64 or non-power-of-two grids). Both halves are linear,
 * so per-GPU grids can be summed over that block alone (178 MB at G 8192,
 * N 5440, against 512 MiB for the whole grid). _finish_rows runs the
 * remaining column passes + screen + correction into dirty_image.
 * scatter + rows + finish_rows == scatter + finish. */
int sdp_gridder_uvw_es_fft_row_spectra(
        const sdp_GridderUvwEsFft* plan,
        int64_t* rows,
        int64_t* col0,
        int64_t* ncols
);
void sdp_grid_uvw_es_fft_rows(
        sdp_GridderUvwEsFft* plan,
        sdp_Mem* grid,
        sdp_Error* status
);
void sdp_grid_uvw_es_fft_finish_rows(
        sdp_GridderUvwEsFft* plan,
        sdp_Mem* grid,
        sdp_Mem* dirty_image,
        sdp_Error* status
);

#ifdef __cplusplus
}
#endif

#endif
