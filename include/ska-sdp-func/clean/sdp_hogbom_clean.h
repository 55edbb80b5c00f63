/* MI355X-native Hogbom CLEAN: drop-in C ABI.
 *
 * Replaces, symbol for symbol and argument for argument,
 *   src/ska-sdp-func/clean/sdp_hogbom_clean.h:36-47
 * of ska-sdp-func 1.2.2 (bound from Python by
 *   src/ska_sdp_func/clean/hogbom_clean.py:7-22).
 *
 * dirty_img     : [N, N] float or double
 * psf           : [2N, 2N], same type
 * cbeam_details : [4] = {BMAJ sigma, BMIN sigma, THETA degrees, SIZE}, float
 *                 or double, host or device (read on the host)
 * clean_model   : [N, N] out: CLEAN components (overwritten)
 * residual      : [N, N] out: dirty image minus the subtracted PSFs
 * skymodel      : [N, N] out: components convolved with the SIZE x SIZE
 *                 Gaussian CLEAN beam ("same"-mode alignment, as
 *                 scipy.signal.convolve and the reference's
 *                 sdp_fft_convolution) plus the residual
 * Each cycle finds the first (lowest flat index) maximum of the residual,
 * stops if it is below threshold, adds loop_gain * peak to the component
 * map and subtracts loop_gain * peak * psf shifted to the peak, at most
 * cycle_limit times; the arithmetic follows the reference CPU path
 * (sdp_hogbom_clean.cpp:183-240: products in double, one rounding to the
 * image type per update), so the components and residual are bit-identical
 * to it. All images on the GPU (asynchronous w.r.t. nothing: the call
 * returns when done) or all on the host (staged through device memory; the
 * computation runs on the GPU).
 */
#ifndef SDP_HOGBOM_CLEAN_H_
#define SDP_HOGBOM_CLEAN_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

void sdp_hogbom_clean(
        const sdp_Mem* dirty_img,
        const sdp_Mem* psf,
        const sdp_Mem* cbeam_details,
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
