/* MI355X-native tiling / bucket sort of visibilities: drop-in C ABI.
 *
 * Replaces, symbol for symbol and argument for argument,
 *   src/ska-sdp-func/visibility/sdp_tiled_functions.h:62-76 (count and
 *   prefix sum), :136-153 (bucket sort), :200-217 (tiled indexing)
 * of ska-sdp-func 1.2.2 (bound from Python by
 *   src/ska_sdp_func/visibility/tiled_functions.py).
 *
 * Semantics are those of the reference GPU kernels
 * (sdp_tiled_functions.cu:63-291): a visibility at grid cell (gu, gv) with
 * gu, gv in [support, grid_size - support) is listed in every tile
 * (pu, pv) with pu in [floor((gu - top_left_u - support) / tile_u),
 * ceil((gu - top_left_u + support + 1) / tile_u)) (float arithmetic) and
 * likewise for v; tile index pu + pv * num_tiles_u; sorted_tile = pv * 32768
 * + pu; sorted_vis / sorted_weight take element (t, b, c) of the vis /
 * weight arrays read as real arrays of the uvw precision, as the reference
 * kernel indexes them. Differences, on purpose: entries within a tile are
 * in visibility order (t, b, c) -- deterministic, where the reference's
 * atomics leave the order arbitrary; tile indices outside [0, num_tiles)
 * (which the reference writes out of bounds) are dropped. All arrays must
 * be on the GPU (SDP_ERR_MEM_LOCATION otherwise): the reference CPU path
 * calls its tile-range macro with the u-minimum slot bound to tile_v_min
 * (sdp_tiled_functions.cpp:84-89), so it computes a different function.
 * Integer outputs are int32.
 */
#ifndef SDP_TILED_FUNCTIONS_H_
#define SDP_TILED_FUNCTIONS_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

void sdp_count_and_prefix_sum(
        const sdp_Mem* uvw,
        const sdp_Mem* freqs,
        const sdp_Mem* vis,
        const int grid_size,
        const int64_t tile_size_u,
        const int64_t tile_size_v,
        const double cell_size_rad,
        const int64_t support,
        int* num_visibilites,
        sdp_Mem* tile_offsets,
        sdp_Mem* num_points_in_tiles,
        sdp_Mem* num_skipped,
        sdp_Error* status
);

void sdp_bucket_sort(
        const sdp_Mem* uvw,
        const sdp_Mem* freqs,
        const sdp_Mem* vis,
        const sdp_Mem* weights,
        const int grid_size,
        const int64_t tile_size_u,
        const int64_t tile_size_v,
        const double cell_size_rad,
        const int64_t support,
        sdp_Mem* sorted_uu,
        sdp_Mem* sorted_vv,
        sdp_Mem* sorted_weight,
        sdp_Mem* sorted_tile,
        sdp_Mem* sorted_vis,
        sdp_Mem* tile_offsets,
        sdp_Error* status
);

void sdp_tiled_indexing(
        const sdp_Mem* uvw,
        const sdp_Mem* freqs,
        const int grid_size,
        const int64_t tile_size_u,
        const int64_t tile_size_v,
        const double cell_size_rad,
        const int64_t support,
        const int64_t num_channels,
        const int64_t num_baselines,
        const int64_t num_times,
        sdp_Mem* sorted_tile,
        sdp_Mem* sorted_uu,
        sdp_Mem* sorted_vv,
        sdp_Mem* sorted_vis_index,
        sdp_Mem* tile_offsets,
        sdp_Error* status
);

#ifdef __cplusplus
}
#endif

#endif
