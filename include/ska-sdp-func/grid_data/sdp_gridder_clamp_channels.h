/* MI355X-native gridder channel clamping: drop-in C ABI.
 *
 * Replaces src/ska-sdp-func/grid_data/sdp_gridder_clamp_channels.h of
 * ska-sdp-func 1.2.2: same include path, function names, arguments and
 * semantics. The two array functions are exported by libska_sdp_func
 * (implementation: ska-sdp-func_amd/csrc/grid_data/sdp_gridder_utils.hip,
 * GPU kernels for device arrays, host arrays staged through HBM); the
 * per-position form is header-only, as in the reference.
 */
#ifndef SDP_GRIDDER_CLAMP_CHANNELS_H_
#define SDP_GRIDDER_CLAMP_CHANNELS_H_

#include "ska-sdp-func/math/sdp_math_macros.h"
#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Restrict per-row channel ranges [start_ch_in, end_ch_in) so that every
 * visibility of rows [start_row, end_row) has min_u <= uvw[dim] * f / c
 * < max_u (ref. sdp_gridder_clamp_channels.h:42-56; impl .cpp:8-62).
 * Rows outside [start_row, end_row) are left untouched in the outputs.
 * uvws [rows, 3] float/double, channel arrays int64 [rows]. */
void sdp_gridder_clamp_channels_single(
        const sdp_Mem* uvws,
        const int dim,
        const double freq0_hz,
        const double dfreq_hz,
        const sdp_Mem* start_ch_in,
        const sdp_Mem* end_ch_in,
        const double min_u,
        const double max_u,
        sdp_Mem* start_ch_out,
        sdp_Mem* end_ch_out,
        int64_t start_row,
        int64_t end_row,
        sdp_Error* status
);

/* Same, in u (dimension 0) then v (dimension 1) (ref.
 * sdp_gridder_clamp_channels.h:79-94; impl .cpp:64-150). */
void sdp_gridder_clamp_channels_uv(
        const sdp_Mem* uvws,
        const double freq0_hz,
        const double dfreq_hz,
        const sdp_Mem* start_ch_in,
        const sdp_Mem* end_ch_in,
        const double min_u,
        const double max_u,
        const double min_v,
        const double max_v,
        sdp_Mem* start_ch_out,
        sdp_Mem* end_ch_out,
        int64_t start_row,
        int64_t end_row,
        sdp_Error* status
);

/* Clamp one row's channel range [*start_ch, *end_ch) to the channels whose
 * coordinate (u in metres scaled by freq0_hz + ch * dfreq_hz, over c) lies
 * in [min_u, max_u) (ref. sdp_gridder_clamp_channels.h:116-172).
 *
 * The coordinate is linear in the channel, x(ch) = x0 + ch * dx, so the
 * bounds are ceil((bound - x0) / dx), swapped when dx < 0. To keep the
 * quotient inside the int64 conversion range, dx is treated as zero when
 * |dx| <= max(|min_u - x0|, |max_u - x0|) / 2147483645; then the range is
 * kept whole or emptied according to whether x0 lies in [min_u, max_u).
 * An empty result is always returned as (0, 0). Start is inclusive and end
 * exclusive, so adjacent boxes sharing a bound never share a channel. */
SDP_INLINE
void sdp_gridder_clamp_channels_inline(
        const double u,
        const double freq0_hz,
        const double dfreq_hz,
        int64_t* start_ch,
        int64_t* end_ch,
        const double min_u,
        const double max_u
)
{
    const double x0 = freq0_hz * u / C_0;
    const double dx = dfreq_hz * u / C_0;
    const double lo_rel = min_u - x0;
    const double hi_rel = max_u - x0;
    const double tiny = MAX(fabs(lo_rel), fabs(hi_rel)) / 2147483645.0;
    if (dx > tiny || dx < -tiny)
    {
        /* Increasing coordinate: [lo, hi) -> [ceil(lo_rel / dx),
         * ceil(hi_rel / dx)); decreasing: the bounds change roles. */
        const double first = (dx > 0.0) ? lo_rel : hi_rel;
        const double last = (dx > 0.0) ? hi_rel : lo_rel;
        const int64_t s = (int64_t)ceil(first / dx);
        const int64_t e = (int64_t)ceil(last / dx);
        if (s > *start_ch) *start_ch = s;
        if (e < *end_ch) *end_ch = e;
    }
    else if (min_u > x0 || max_u <= x0)
    {
        *start_ch = 0;
        *end_ch = 0;
    }
    if (*end_ch <= *start_ch)
    {
        *start_ch = 0;
        *end_ch = 0;
    }
}

#ifdef __cplusplus
}
#endif

#endif /* SDP_GRIDDER_CLAMP_CHANNELS_H_ */
