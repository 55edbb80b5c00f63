/* MI355X-native gridder utilities of the w-towers path: drop-in C ABI.
 *
 * src/ska-sdp-func/grid_data/sdp_gridder_utils.h of ska-sdp-func 1.2.2
 * (the channel clamps are in sdp_gridder_clamp_channels.h, as in the
 * reference); same names, arguments and semantics.
 * Table generators (make_kernel, make_pswf_kernel, make_w_pattern) fill
 * host (CPU) arrays, as in the reference; the array operations run on the
 * GPU for device arrays and stage host arrays through device memory.
 */
#ifndef SDP_GRIDDER_UTILS_H_
#define SDP_GRIDDER_UTILS_H_

#include "ska-sdp-func/math/sdp_math_macros.h"
#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

/* out += in1 * in2 ** exponent (in2 may be NULL: out += in1; a real out
 * takes the real part), sdp_gridder_utils.h:40-46 (impl .cpp:722-852). */
void sdp_gridder_accumulate_scaled_arrays(
        sdp_Mem* out,
        const sdp_Mem* in1,
        const sdp_Mem* in2,
        int exponent,
        sdp_Error* status
);

/* w step for a field of view, .h:69-75 (impl .cpp:1016-1039). */
double sdp_gridder_determine_w_step(
        double theta,
        double fov,
        double shear_u,
        double shear_v,
        double x0
);

/* Oversampled uv kernel [oversampling + 1, support] from an image-space
 * window [support], .h:204-208 (impl .cpp:385-427, 1305-1326). */
void sdp_gridder_make_kernel(
        const sdp_Mem* window,
        sdp_Mem* kernel,
        sdp_Error* status
);

/* PSWF kernel [oversampling + 1, support], .h:221-225 (.cpp:1329-1350). */
void sdp_gridder_make_pswf_kernel(
        int support,
        sdp_Mem* kernel,
        sdp_Error* status
);

/* exp(2 pi i w_step n(l, m)) [subgrid_size, subgrid_size] complex double,
 * .h:240-248 (.cpp:1353-1380). */
void sdp_gridder_make_w_pattern(
        int subgrid_size,
        double theta,
        double shear_u,
        double shear_v,
        double w_step,
        sdp_Mem* w_pattern,
        sdp_Error* status
);

/* sqrt(mean(|a - b|^2)), .h:276-280 (.cpp:1469-1538). */
double sdp_gridder_rms_diff(
        const sdp_Mem* a,
        const sdp_Mem* b,
        sdp_Error* status
);

/* out = in1 / in2 ** exponent, .h:296-302 (.cpp:1541-1667). */
void sdp_gridder_scale_inv_array(
        sdp_Mem* out,
        const sdp_Mem* in1,
        const sdp_Mem* in2,
        int exponent,
        sdp_Error* status
);

/* subgrids[:-1] = subgrids[1:], .h:310 (.cpp:1670-1726). */
void sdp_gridder_shift_subgrids(sdp_Mem* subgrids, sdp_Error* status);

/* grid (periodically wrapped) += factor * subgrid at -offset,
 * .h:322-329 (.cpp:553-601, 1729-1822). */
void sdp_gridder_subgrid_add(
        sdp_Mem* grid,
        int offset_u,
        int offset_v,
        const sdp_Mem* subgrid,
        double factor,
        sdp_Error* status
);

/* subgrid = grid at offset (periodic), .h:340-346 (.cpp:603-649). */
void sdp_gridder_subgrid_cut_out(
        const sdp_Mem* grid,
        int offset_u,
        int offset_v,
        sdp_Mem* subgrid,
        sdp_Error* status
);

/* result = sum(a[start:end] - b[start:end]), int32 arrays; start < 0 or
 * end < 0: all rows. .h:358-365 (.cpp:652-679, 1919-1989). */
void sdp_gridder_sum_diff(
        const sdp_Mem* a,
        const sdp_Mem* b,
        int64_t* result,
        int64_t start_row,
        int64_t end_row,
        sdp_Error* status
);

/* Scaled uvw bounding box of the selected channels, starting from 0 in
 * every dimension, .h:379-388 (.cpp:682-719, 1992-2102). */
void sdp_gridder_uvw_bounds_all(
        const sdp_Mem* uvws,
        double freq0_hz,
        double dfreq_hz,
        const sdp_Mem* start_chs,
        const sdp_Mem* end_chs,
        double uvw_min[3],
        double uvw_max[3],
        sdp_Error* status
);

/* Number of non-zero pixels (complex: either part) of a 2-D image of
 * shape[0] rows, .h:54-57 (impl .cpp:106-123, 987-1013). Runs on the GPU
 * (host images are staged). */
int64_t sdp_gridder_count_nonzero_pixels(
        const sdp_Mem* image,
        sdp_Error* status
);

/* vis[i, c] += sum_s flux[s] exp(-2 pi i (l u + m v + n w)) with (u, v, w)
 * the row's coordinates in wavelengths at channel c minus the sub-grid
 * offsets / theta (w: offset * w_step); a row is skipped when start_chs
 * and end_chs are given and start >= end. Types: double lmn / uvw, complex
 * double vis, or the float triple; flux double. .h:99-114 (impl
 * .cpp:126-212, 1042-1100). Runs on the GPU. */
void sdp_gridder_dft(
        const sdp_Mem* uvws,
        const sdp_Mem* start_chs,
        const sdp_Mem* end_chs,
        const sdp_Mem* flux,
        const sdp_Mem* lmn,
        int subgrid_offset_u,
        int subgrid_offset_v,
        int subgrid_offset_w,
        double theta,
        double w_step,
        double freq0_hz,
        double dfreq_hz,
        sdp_Mem* vis,
        sdp_Error* status
);

/* image[il, im] += taper[il] taper[im] sum_(i, c) vis[i, c]
 * exp(+2 pi i (l u + m v + n w)) with lmn[il * size + im] the pixel's
 * direction cosines (complex image, same precision as vis / uvw / lmn).
 * .h:140-156 (impl .cpp:215-314, 1103-1239). Runs on the GPU. */
void sdp_gridder_idft(
        const sdp_Mem* uvws,
        const sdp_Mem* vis,
        const sdp_Mem* start_chs,
        const sdp_Mem* end_chs,
        const sdp_Mem* lmn,
        const sdp_Mem* image_taper_1d,
        int subgrid_offset_u,
        int subgrid_offset_v,
        int subgrid_offset_w,
        double theta,
        double w_step,
        double freq0_hz,
        double dfreq_hz,
        sdp_Mem* image,
        sdp_Error* status
);

/* (l, m, n) of every pixel (flux NULL) or of the non-zero pixels with
 * their (tapered) real values in flux; l = (il - size / 2) theta / size.
 * Host (CPU) output tables, as in the reference. .h:181-190 (impl
 * .cpp:317-382, 1242-1302). */
void sdp_gridder_image_to_flmn(
        const sdp_Mem* image,
        double theta,
        double shear_u,
        double shear_v,
        const sdp_Mem* image_taper_1d,
        sdp_Mem* flux,
        sdp_Mem* lmn,
        sdp_Error* status
);

/* out = a - b (out in CPU memory, same type as a), .h:260-265 (impl
 * .cpp:429-458, 1383-1466). */
void sdp_gridder_residual(
        const sdp_Mem* a,
        const sdp_Mem* b,
        sdp_Mem* out,
        sdp_Error* status
);

#ifdef __cplusplus
}
#endif

#endif
