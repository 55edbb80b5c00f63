/* MI355X-native visibility weighting (uniform and Briggs/robust): drop-in
 * C ABI.
 *
 * Replaces, symbol for symbol and argument for argument,
 *   src/ska-sdp-func/visibility/sdp_weighting.h:50-69
 * of ska-sdp-func 1.2.2 (bound from Python by
 *   src/ska_sdp_func/visibility/weighting.py:11-38).
 *
 * uvw            : [num_times, num_baselines, 3] real (metres)
 * freq_hz        : [num_channels] real
 * weight_grid_uv : [grid_size, grid_size, num_pols] real, accumulated into
 *                  (the caller zero-initialises it, as in the reference)
 * input_weights  : [num_times, num_baselines, num_channels, num_pols] real
 * output_weights : same shape and type; written only for visibilities whose
 *                  cell lies on the grid (others keep their content)
 * Cell of a visibility (sdp_weighting.cpp:46-53):
 *   idx = (int64)(floor(uv f / c / max_abs_uv * (grid_size / 2))
 *                 + grid_size / 2)
 * Uniform: out = 1 / grid[cell]; Briggs: out = in / (1 + R grid[cell]),
 * R = (5 10^-robust)^2 / (sum_vis grid^2 / sum_vis grid) (:143-154).
 *
 * Types (as the reference): uvw and freq_hz double; input/output weights
 * and the grid both double or both float. Any other combination gives
 * SDP_ERR_DATA_TYPE "Unsupported data type(s)". Location: all arrays on the
 * GPU (computed asynchronously on the null stream), or all on the host --
 * then they are staged through device memory (the computation runs on the
 * GPU). Differences from the reference: cells with a negative index (the
 * reference writes before the grid, undefined behaviour) are skipped like
 * cells past the end; grid sums are accumulated with device atomics
 * (summation order differs, ~1e-16 relative in double).
 */
#ifndef SDP_WEIGHTING_H_
#define SDP_WEIGHTING_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

void sdp_weighting_briggs(
        const sdp_Mem* uvw,
        const sdp_Mem* freq_hz,
        double max_abs_uv,
        const double robust_param,
        sdp_Mem* weight_grid_uv,
        sdp_Mem* input_weights,
        sdp_Mem* output_weights,
        sdp_Error* status
);

void sdp_weighting_uniform(
        const sdp_Mem* uvw,
        const sdp_Mem* freq_hz,
        double max_abs_uv,
        sdp_Mem* weight_grid_uv,
        sdp_Mem* input_weights,
        sdp_Mem* output_weights,
        sdp_Error* status
);

#ifdef __cplusplus
}
#endif

#endif
