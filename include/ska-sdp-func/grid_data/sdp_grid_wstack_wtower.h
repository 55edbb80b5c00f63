/* MI355X-native w-stacking x w-towers imaging driver: drop-in C ABI.
 *
 * Replaces src/ska-sdp-func/grid_data/sdp_grid_wstack_wtower.h:44-109 of
 * ska-sdp-func 1.2.2 (bound from Python by
 * src/ska_sdp_func/grid_data/grid_wstack_wtower.py:146-196).
 *
 * Same arguments and results as the reference: every visibility is
 * assigned to the same (w-stack plane, sub-grid, w-layer) as the
 * reference's channel clamps assign it, and is (de)gridded with the same
 * PSWF kernels, w-pattern algebra and corrections. The execution differs:
 * the reference scans all rows once per sub-grid (O(rows x sub-grids)) and
 * runs one sub-grid task at a time; here one device pass bins the
 * visibilities by (w-stack plane, sub-grid, w-layer) and all sub-grids of
 * a w-stack plane move through their w-towers together, with batched
 * FFTs. Results agree with the reference up to floating-point summation
 * order.
 *
 * Arrays may be in CPU or GPU memory (all in the same place); CPU arrays
 * are staged through device memory and the work runs on the GPU.
 * num_threads is accepted and ignored (the reference uses 1 on GPUs).
 * Type combinations (vis / uvw): c128 / f64, c64 / f64, c64 / f32; the
 * image may be real or complex, single or double precision.
 */
#ifndef SDP_GRID_WSTACK_WTOWER_H_
#define SDP_GRID_WSTACK_WTOWER_H_

#include <stdint.h>

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

/* image (zeroed first) = gridded visibilities, .h:44-73
 * (impl sdp_grid_wstack_wtower.cpp:475-736). */
void sdp_grid_wstack_wtower_grid_all(
        const sdp_Mem* vis,
        double freq0_hz,
        double dfreq_hz,
        const sdp_Mem* uvw,
        int subgrid_size,
        double theta,
        double w_step,
        double shear_u,
        double shear_v,
        int support,
        int oversampling,
        int w_support,
        int w_oversampling,
        double subgrid_frac,
        double w_tower_height,
        int verbosity,
        sdp_Mem* image,
        int num_threads,
        sdp_Error* status
);

/* vis (zeroed first) = degridded image, .h:80-109
 * (impl sdp_grid_wstack_wtower.cpp:218-472). */
void sdp_grid_wstack_wtower_degrid_all(
        const sdp_Mem* image,
        double freq0_hz,
        double dfreq_hz,
        const sdp_Mem* uvw,
        int subgrid_size,
        double theta,
        double w_step,
        double shear_u,
        double shear_v,
        int support,
        int oversampling,
        int w_support,
        int w_oversampling,
        double subgrid_frac,
        double w_tower_height,
        int verbosity,
        sdp_Mem* vis,
        int num_threads,
        sdp_Error* status
);

/* MI355X extension (not in the reference): the same operations restricted
 * to the w-stack planes iw with (iw - min_iw) % plane_stride ==
 * plane_offset, where min_iw is the lowest plane of the data. Used to
 * shard w-stack planes across GPUs (one process per GPU): the images of
 * all shards sum to the grid_all image; the visibilities of all shards
 * sum to the degrid_all visibilities. plane_stride = 1, plane_offset = 0
 * is grid_all / degrid_all. The output is still zeroed first. */
void sdp_grid_wstack_wtower_grid_planes(
        const sdp_Mem* vis,
        double freq0_hz,
        double dfreq_hz,
        const sdp_Mem* uvw,
        int subgrid_size,
        double theta,
        double w_step,
        double shear_u,
        double shear_v,
        int support,
        int oversampling,
        int w_support,
        int w_oversampling,
        double subgrid_frac,
        double w_tower_height,
        int verbosity,
        sdp_Mem* image,
        int plane_offset,
        int plane_stride,
        sdp_Error* status
);

void sdp_grid_wstack_wtower_degrid_planes(
        const sdp_Mem* image,
        double freq0_hz,
        double dfreq_hz,
        const sdp_Mem* uvw,
        int subgrid_size,
        double theta,
        double w_step,
        double shear_u,
        double shear_v,
        int support,
        int oversampling,
        int w_support,
        int w_oversampling,
        double subgrid_frac,
        double w_tower_height,
        int verbosity,
        sdp_Mem* vis,
        int plane_offset,
        int plane_stride,
        sdp_Error* status
);

/* MI355X extension: the same operations restricted to an explicit set of
 * w-stack planes, for load-balanced sharding across GPUs. Plane iw is the
 * reference's w-stack plane index (w f / c in [iw d - d/2, (iw + 1) d -
 * d/2), d = w_tower_height * w_step, sdp_grid_wstack_wtower.cpp:336-343);
 * it is processed iff plane_mask[clamp(iw - plane_first, 0, n - 1)] != 0,
 * plane_mask a 1-D int32 array of n entries (host or device): planes below
 * plane_first belong to the owner of entry 0, planes past the range to the
 * owner of entry n - 1. Disjoint masks covering the n entries therefore
 * cover every plane, and give images / visibilities that sum to the
 * grid_all / degrid_all ones even where the caller's plane-range model
 * misses a plane. */
void sdp_grid_wstack_wtower_grid_plane_set(
        const sdp_Mem* vis,
        double freq0_hz,
        double dfreq_hz,
        const sdp_Mem* uvw,
        int subgrid_size,
        double theta,
        double w_step,
        double shear_u,
        double shear_v,
        int support,
        int oversampling,
        int w_support,
        int w_oversampling,
        double subgrid_frac,
        double w_tower_height,
        int verbosity,
        sdp_Mem* image,
        int64_t plane_first,
        const sdp_Mem* plane_mask,
        sdp_Error* status
);

void sdp_grid_wstack_wtower_degrid_plane_set(
        const sdp_Mem* image,
        double freq0_hz,
        double dfreq_hz,
        const sdp_Mem* uvw,
        int subgrid_size,
        double theta,
        double w_step,
        double shear_u,
        double shear_v,
        int support,
        int oversampling,
        int w_support,
        int w_oversampling,
        double subgrid_frac,
        double w_tower_height,
        int verbosity,
        sdp_Mem* vis,
        int64_t plane_first,
        const sdp_Mem* plane_mask,
        sdp_Error* status
);

/* Device timing of the fused tower kernels (k_tower_dft when gridding,
 * k_tower_idft when degridding) accumulated over the calls made while
 * enabled: HIP events around every launch. enable_timing(1) switches it on
 * and resets the totals; get_timing writes up to max_values of
 * [0] total kernel time (ms), [1] launches, [2] visibilities gridded or
 * degridded by the fused kernels, [3] sub-grid w-layers they stepped
 * through, [4] sub-grid size, [5] 0 gridding / 1 degridding (last call)
 * and returns the number written (0 if timing is off). Extension with no
 * reference counterpart: the reference has no device path to time. */
void sdp_grid_wstack_wtower_enable_timing(int enable);
int sdp_grid_wstack_wtower_get_timing(double* out, int max_values);

#ifdef __cplusplus
}
#endif

#endif
