/* MI355X-native dynamic-threshold RFI flagger: drop-in C ABI.
 *
 * Replaces, symbol for symbol and argument for argument,
 *   src/ska-sdp-func/visibility/sdp_flagger.h:53-64
 * of ska-sdp-func 1.2.2 (bound from Python by
 *   src/ska_sdp_func/visibility/flagger.py:10-25).
 *
 * vis  : [num_timesamples, num_baselines, num_channels, num_pols] complex
 *        (c64 or c128), C-contiguous;
 * flags: int32, same shape, C-contiguous, writable; flags are only ever SET
 *        to 1 (existing content is kept), as in the reference.
 * Results are bit-identical to the reference CPU function
 * (sdp_flagger.cpp:125-428) for every supported shape, including its
 * quirks (upper-middle "median", variation MAD around the magnitude median,
 * channel 0 never flagged as a window neighbour, t - 1 flagged by the
 * variation test).
 *
 * Location: both arrays on the GPU (computed in place, asynchronously on
 * the null stream), or both on the host -- then they are staged through
 * device memory (the computation still runs on the GPU). Limits of this
 * implementation: num_channels <= 2048, window_median_history <= 1024,
 * 1 <= sampling_step <= num_channels (SDP_ERR_INVALID_ARGUMENT otherwise).
 * Positions are 64-bit: arrays beyond 2^31 elements are handled (the
 * reference's int positions overflow there; it must be called per chunk of
 * baselines, with identical results).
 */
#ifndef SDP_FLAGGER_H_
#define SDP_FLAGGER_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

/* sdp_flagger.h:53-64 (impl sdp_flagger.cpp:351-428) */
void sdp_flagger_dynamic_threshold(
        const sdp_Mem* vis,
        sdp_Mem* flags,
        const double alpha,
        const double threshold_magnitudes,
        const double threshold_variations,
        const double threshold_broadband,
        const int sampling_step,
        const int window,
        const int window_median_history,
        sdp_Error* status
);

#ifdef __cplusplus
}
#endif

#endif
