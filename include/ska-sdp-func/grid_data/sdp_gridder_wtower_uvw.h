/* MI355X-native w-towers sub-grid (de)gridder: drop-in C ABI.
 *
 * Replaces, symbol for symbol and argument for argument,
 *   src/ska-sdp-func/grid_data/sdp_gridder_wtower_uvw.h:59-285
 * of ska-sdp-func 1.2.2 (bound from Python by
 *   src/ska_sdp_func/grid_data/gridder_wtower_uvw.py:425-575).
 *
 * Semantics kept from the reference (sdp_gridder_wtower_uvw.cpp): a stack
 * of w_support sub-grids is moved through the w-planes of the data by FFT
 * and multiplication with the w-pattern; visibilities are (de)gridded with
 * oversampled PSWF kernels in (u, v) and w; degrid accumulates into vis,
 * grid accumulates into subgrid_image; start_row < 0 or end_row < 0 means
 * all rows; dfreq_hz == 0 is replaced by 10 Hz.
 *
 * Type combinations (subgrid / uvws / vis): c128/f64/c128, c64/f64/c64,
 * c64/f32/c64. Device arrays are processed on the GPU (asynchronously on
 * the null stream); host arrays are staged through device memory (the work
 * still runs on the GPU). All arrays of a call must share one location.
 *
 * The PSWF is evaluated from its Legendre expansion (lowest eigenvector of
 * the prolate operator) rather than the reference's specfun port; values
 * agree to ~1e-13 relative for support <= 10 (tests/test_wtower_oracle.py).
 */
#ifndef SDP_GRIDDER_WTOWER_UVW_H_
#define SDP_GRIDDER_WTOWER_UVW_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

struct sdp_GridderWtowerUVW;
typedef struct sdp_GridderWtowerUVW sdp_GridderWtowerUVW;

/* sdp_gridder_wtower_uvw.h:59-71 (impl .cpp:660-723) */
sdp_GridderWtowerUVW* sdp_gridder_wtower_uvw_create(
        int image_size,
        int subgrid_size,
        double theta,
        double w_step,
        double shear_u,
        double shear_v,
        int support,
        int oversampling,
        int w_support,
        int w_oversampling,
        sdp_Error* status
);

/* .h:93-108 (impl .cpp:726-909) */
void sdp_gridder_wtower_uvw_degrid(
        sdp_GridderWtowerUVW* plan,
        const sdp_Mem* subgrid_image,
        int subgrid_offset_u,
        int subgrid_offset_v,
        int subgrid_offset_w,
        double freq0_hz,
        double dfreq_hz,
        const sdp_Mem* uvws,
        const sdp_Mem* start_chs,
        const sdp_Mem* end_chs,
        sdp_Mem* vis,
        int64_t start_row,
        int64_t end_row,
        sdp_Error* status
);

/* .h:119-126 (impl .cpp:912-932) */
void sdp_gridder_wtower_uvw_degrid_correct(
        sdp_GridderWtowerUVW* plan,
        sdp_Mem* facet,
        int facet_offset_l,
        int facet_offset_m,
        int w_offset,
        sdp_Error* status
);

/* .h:150-165 (impl .cpp:935-1123) */
void sdp_gridder_wtower_uvw_grid(
        sdp_GridderWtowerUVW* plan,
        const sdp_Mem* vis,
        const sdp_Mem* uvws,
        const sdp_Mem* start_chs,
        const sdp_Mem* end_chs,
        double freq0_hz,
        double dfreq_hz,
        sdp_Mem* subgrid_image,
        int subgrid_offset_u,
        int subgrid_offset_v,
        int subgrid_offset_w,
        int64_t start_row,
        int64_t end_row,
        sdp_Error* status
);

/* .h:176-183 (impl .cpp:1126-1146) */
void sdp_gridder_wtower_uvw_grid_correct(
        sdp_GridderWtowerUVW* plan,
        sdp_Mem* facet,
        int facet_offset_l,
        int facet_offset_m,
        int w_offset,
        sdp_Error* status
);

/* .h:189 (impl .cpp:1149-1159) */
void sdp_gridder_wtower_uvw_free(sdp_GridderWtowerUVW* plan);

/* .h:196-199: w-planes processed so far; gridding = 0 degrid, 1 grid. */
int sdp_gridder_wtower_uvw_num_w_planes(
        const sdp_GridderWtowerUVW* plan,
        int gridding
);

/* Accessors, .h:206-285. */
int sdp_gridder_wtower_uvw_image_size(const sdp_GridderWtowerUVW* plan);
int sdp_gridder_wtower_uvw_oversampling(const sdp_GridderWtowerUVW* plan);
double sdp_gridder_wtower_uvw_shear_u(const sdp_GridderWtowerUVW* plan);
double sdp_gridder_wtower_uvw_shear_v(const sdp_GridderWtowerUVW* plan);
int sdp_gridder_wtower_uvw_subgrid_size(const sdp_GridderWtowerUVW* plan);
int sdp_gridder_wtower_uvw_support(const sdp_GridderWtowerUVW* plan);
double sdp_gridder_wtower_uvw_theta(const sdp_GridderWtowerUVW* plan);
int sdp_gridder_wtower_uvw_w_oversampling(const sdp_GridderWtowerUVW* plan);
double sdp_gridder_wtower_uvw_w_step(const sdp_GridderWtowerUVW* plan);
int sdp_gridder_wtower_uvw_w_support(const sdp_GridderWtowerUVW* plan);

#ifdef __cplusplus
}
#endif

#endif
