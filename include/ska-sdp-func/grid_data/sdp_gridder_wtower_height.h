/* MI355X-native w-tower height search: drop-in C ABI.
 *
 * Replaces src/ska-sdp-func/grid_data/sdp_gridder_wtower_height.h:43-77 of
 * ska-sdp-func 1.2.2 (bound from Python by
 * src/ska_sdp_func/grid_data/gridder_utils.py:118-245, 389-541).
 *
 * The accuracy probe (worst-case image -> degrid_correct -> FFT -> cut-out
 * -> inverse FFT -> w-towers degrid at sampled (u, v, w)) runs on the GPU;
 * the direct Fourier sum it is compared with (9 rows x 4 sources by
 * default) is evaluated on the host, as in the reference.
 */
#ifndef SDP_GRIDDER_WTOWER_HEIGHT_H_
#define SDP_GRIDDER_WTOWER_HEIGHT_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Maximum w-tower height (in units of w_step) for which degridding at
 * height w stays within target_err of the DFT (target_err = 0: twice the
 * error at w = 0). subgrid_frac = 0 means 2/3; num_samples = 0 means 3.
 * Reference .h:43-59 (impl .cpp:187-269). */
double sdp_gridder_determine_max_w_tower_height(
        int image_size,
        int subgrid_size,
        double theta,
        double w_step,
        double shear_u,
        double shear_v,
        int support,
        int oversampling,
        int w_support,
        int w_oversampling,
        double fov,
        double subgrid_frac,
        int num_samples,
        double target_err,
        sdp_Error* status
);

/* Four point sources at the edge of the field of view in a square complex
 * double CPU image, .h:71-77 (impl .cpp:272-316). */
void sdp_gridder_worst_case_image(
        double theta,
        double fov,
        sdp_Mem* image,
        sdp_Error* status
);

#ifdef __cplusplus
}
#endif

#endif
