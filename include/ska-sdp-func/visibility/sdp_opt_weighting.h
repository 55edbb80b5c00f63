/* MI355X-native tiled Briggs weighting: drop-in C ABI.
 *
 * Replaces, symbol for symbol and argument for argument,
 *   src/ska-sdp-func/visibility/sdp_opt_weighting.h:71-87 (bucket form)
 *   src/ska-sdp-func/visibility/sdp_opt_weighting.h:124-141 (indexed form)
 * of ska-sdp-func 1.2.2 (bound from Python by
 *   src/ska_sdp_func/visibility/opt_weighting.py:7-50).
 *
 * Inputs are the outputs of sdp_count_and_prefix_sum followed by
 * sdp_bucket_sort (bucket form) or sdp_tiled_indexing (indexed form),
 * tile size 32 x 16 (fixed, as the reference .cpp:48-49). Workgroup b
 * (b < num_tiles - 1, as the reference launch .cpp:123) takes the run
 * [tile_offsets[b], tile_offsets[b + 1]) of the sorted arrays -- after the
 * sort advanced the cursors, the entries of tile b + 1 -- decodes its tile
 * from sorted_tile[run start] (u = code & 32767, v = code >> 15) and, for
 * the entries whose cell (round(sorted_uu) + grid_size / 2, likewise v)
 * lies inside that tile (an entry is listed in every tile its support
 * touches, and counts only in its own):
 *   W[cell]   = sum of the entries' weights in the cell;
 *   sw, sw2   = sum over those entries of W[cell], W[cell]^2;
 *   R         = (5 10^-robust_param)^2 / (sw2 / sw);
 *   out       = weight / (1 + R W[cell]),
 * written to output_weights[entry position] (bucket form, weights taken
 * from sorted_weight) or output_weights[sorted_vis_index[entry]] (indexed
 * form, weights[sorted_vis_index[entry]]). Other output elements are left
 * untouched.
 *
 * Differences from the reference kernels (sdp_opt_weighting.cu:21-275),
 * each a defect of the reference that makes its output depend on
 * scheduling; the reference's own test (tests/visibility/
 * test_opt_weighting.py) calls the bucket form "inaccurate ... not tested"
 * and checks the indexed form against a global Briggs weighting, which the
 * per-tile result above equals on its one-tile data set:
 *   - the loops run to the end of the run (the reference compares the
 *     absolute index with the run length, .cu:56, :166);
 *   - R is formed after all of sw / sw2 are summed (the reference forms it
 *     inside the summing loop, racing the other threads' atomics, .cu:96);
 *   - sw and sw2 are separate sums (the indexed kernel declares them as
 *     three extern shared arrays that alias the cell table, .cu:155-157);
 *   - robust_param is used as the double passed (the kernels declare an
 *     int parameter and receive the low 32 bits of the double, .cu:33);
 *   - cell sums use device double atomics, so their rounding (not their
 *     value for integer weights) depends on order, as in the reference.
 *
 * Types (as the reference): uvw, weights, sorted positions and weights
 * double; sorted_tile, tile_offsets, sorted_vis_index int32. Arrays on the
 * host give SDP_ERR_MEM_LOCATION ("CPU Briggs Weighting doesn't exist
 * yet!") for double data and SDP_ERR_DATA_TYPE otherwise, as the
 * reference (.cpp:96-108). Runs on the null stream.
 */
#ifndef SDP_OPT_WEIGHTING_H_
#define SDP_OPT_WEIGHTING_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

void sdp_optimized_weighting(
        const sdp_Mem* uvw,
        const sdp_Mem* freqs,
        const sdp_Mem* vis,
        const sdp_Mem* weights,
        const double robust_param,
        const int grid_size,
        const int64_t support,
        sdp_Mem* sorted_uu,
        sdp_Mem* sorted_vv,
        sdp_Mem* sorted_weight,
        sdp_Mem* sorted_tile,
        sdp_Mem* tile_offsets,
        sdp_Mem* num_points_in_tiles,
        sdp_Mem* output_weights,
        sdp_Error* status
);

void sdp_optimised_indexed_weighting(
        const sdp_Mem* uvw,
        const sdp_Mem* vis,
        const sdp_Mem* weights,
        const double robust_param,
        const int grid_size,
        const double cell_size_rad,
        const int64_t support,
        const int* num_visibilites,
        sdp_Mem* sorted_tile,
        sdp_Mem* sorted_uu,
        sdp_Mem* sorted_vv,
        sdp_Mem* sorted_vis_index,
        sdp_Mem* tile_offsets,
        sdp_Mem* num_points_in_tiles,
        sdp_Mem* output_weights,
        sdp_Error* status
);

#ifdef __cplusplus
}
#endif

#endif /* SDP_OPT_WEIGHTING_H_ */
