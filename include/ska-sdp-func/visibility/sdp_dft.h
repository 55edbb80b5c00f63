/* MI355X-native point-source DFT prediction: drop-in C ABI.
 *
 * Replaces, symbol for symbol and argument for argument,
 *   src/ska-sdp-func/visibility/sdp_dft.h:47-53 (v00) and :79-87 (v01)
 * of ska-sdp-func 1.2.2 (bound from Python by
 *   src/ska_sdp_func/visibility/dft.py:9-35).
 *
 * source_directions : [components, 3] double (l, m, n as supplied)
 * source_fluxes     : [components, channels, pols] complex double
 * uvw_lambda (v00)  : [times, baselines, channels, 3] double, wavelengths
 * uvw (v01)         : [times, baselines, 3] double, metres; channel c at
 *                     channel_start_hz + c channel_step_hz
 * vis               : [times, baselines, channels, pols] complex double or
 *                     complex float, pols <= 4, overwritten:
 *   vis = sum_s flux[s][c][p] exp(-2 pi i f/c (l u + m v + n w))
 * The phase is formed in double as the reference (sdp_dft.cpp:56-57,
 * :299-300); the phasor is rounded to the visibility precision before the
 * complex multiply-accumulate. Location: all arrays on the GPU
 * (asynchronous, null stream) or all on the host (staged through device
 * memory; the computation runs on the GPU). Type combinations other than
 * the reference's give SDP_ERR_DATA_TYPE.
 */
#ifndef SDP_DFT_H_
#define SDP_DFT_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

void sdp_dft_point_v00(
        const sdp_Mem* source_directions,
        const sdp_Mem* source_fluxes,
        const sdp_Mem* uvw_lambda,
        sdp_Mem* vis,
        sdp_Error* status
);

void sdp_dft_point_v01(
        const sdp_Mem* source_directions,
        const sdp_Mem* source_fluxes,
        const sdp_Mem* uvw,
        const double channel_start_hz,
        const double channel_step_hz,
        sdp_Mem* vis,
        sdp_Error* status
);

#ifdef __cplusplus
}
#endif

#endif
