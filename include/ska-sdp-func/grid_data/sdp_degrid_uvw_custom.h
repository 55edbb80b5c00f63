/* MI355X-native degridding with caller-supplied kernels: drop-in C ABI.
 *
 * Replaces, symbol for symbol and argument for argument,
 *   src/ska-sdp-func/grid_data/sdp_degrid_uvw_custom.h:34-46
 * of ska-sdp-func 1.2.2 (bound from Python by
 *   src/ska_sdp_func/grid_data/degrid_uvw_custom.py:71-88).
 *
 * grid      : [chan][w][v][u][pol] complex double
 * uvw       : [time][baseline][3] double (metres)
 * uv_kernel : [oversampling][stride] double; w_kernel likewise
 * vis       : [time][baseline][chan][pol] complex double, pol 1 or 4;
 *             written for visibilities whose kernel footprint lies strictly
 *             inside the grid (others keep their content), conjugated if
 *             conjugate != 0.
 * Coordinates follow sdp_degrid_uvw_custom.cpp:20-62 (C round, half away
 * from zero); vis = sum_z kw[z] sum_y kv[y] sum_x ku[x] grid[c][z][y][x].
 * Only double precision, as the reference (SDP_ERR_DATA_TYPE otherwise).
 * Location: all arrays on the GPU (asynchronous, null stream) or all on
 * the host (staged through device memory; the computation runs on the
 * GPU). The sums are formed per lane and reduced across the wavefront, so
 * they differ from the reference's sequential order by rounding only.
 */
#ifndef SDP_DEGRID_UVW_CUSTOM_H_
#define SDP_DEGRID_UVW_CUSTOM_H_

#include <stdint.h>

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

void sdp_degrid_uvw_custom(
        const sdp_Mem* grid,
        const sdp_Mem* uvw,
        const sdp_Mem* uv_kernel,
        const sdp_Mem* w_kernel,
        const double theta,
        const double wstep,
        const double channel_start_hz,
        const double channel_step_hz,
        const int32_t conjugate,
        sdp_Mem* vis,
        sdp_Error* status
);

#ifdef __cplusplus
}
#endif

#endif
