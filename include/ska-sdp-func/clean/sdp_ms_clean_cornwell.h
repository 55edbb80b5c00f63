/* MI355X-native multi-scale CLEAN (Cornwell 2008): drop-in C ABI.
 *
 * Replaces, symbol for symbol and argument for argument,
 *   src/ska-sdp-func/clean/sdp_ms_clean_cornwell.h:41-53
 * of ska-sdp-func 1.2.2 (bound from Python by
 *   src/ska_sdp_func/clean/ms_clean_cornwell.py).
 *
 * dirty_img     : [N, N] float or double
 * psf           : [2N, 2N], same type
 * cbeam_details : [4] = {BMAJ sigma, BMIN sigma, THETA degrees, SIZE}; as in
 *                 the reference the beam table is psf-sized and SIZE unused
 * scale_list    : [S] int32 scales in pixels (0 = point), 1 <= S <= 16
 * clean_model   : [N, N] out: CLEAN components (overwritten)
 * residual      : [N, N] out: the scale-0 scaled residual
 * skymodel      : [N, N] out: components (*) beam + residual
 * The reference implements only a CPU path; this one runs on the GPU for
 * host arrays (staged through device memory) and device arrays alike.
 * Convolutions follow the reference's sdp_fft_convolution ("same"
 * alignment), the minor cycle its arithmetic in the image type.
 */
#ifndef SDP_MS_CLEAN_CORNWELL_H_
#define SDP_MS_CLEAN_CORNWELL_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

void sdp_ms_clean_cornwell(
        const sdp_Mem* dirty_img,
        const sdp_Mem* psf,
        const sdp_Mem* cbeam_details,
        const sdp_Mem* scale_list,
        const double loop_gain,
        const double threshold,
        const int cycle_limit,
        sdp_Mem* clean_model,
        sdp_Mem* residual,
        sdp_Mem* skymodel,
        sdp_Error* status
);

#ifdef __cplusplus
}
#endif

#endif
