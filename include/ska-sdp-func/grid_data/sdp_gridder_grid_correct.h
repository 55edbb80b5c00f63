/* Image-plane grid correction of the w-towers path: drop-in C ABI.
 *
 * Replaces src/ska-sdp-func/grid_data/sdp_gridder_grid_correct.h:31-72 of
 * ska-sdp-func 1.2.2 (impl sdp_gridder_grid_correct.cpp:18-326, kernels
 * sdp_gridder_grid_correct.cu:15, :54). Runs on the GPU; host facets are
 * staged through device memory.
 */
#ifndef SDP_GRIDDER_GRID_CORRECT_H_
#define SDP_GRIDDER_GRID_CORRECT_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

/* facet(l, m) /= pswf(l) pswf(m) pswf_n(n) with pswf of c = support pi / 2
 * (values on image_size points, end-corrected) and pswf_n of
 * c = w_support pi / 2 at |2 w_step n| (1 outside |x| < 1); real or
 * complex, float or double facets. .h:31-43. Facet pixels outside the
 * image (undefined in the reference) are left unchanged. */
void sdp_gridder_grid_correct_pswf(
        int image_size,
        double theta,
        double w_step,
        double shear_u,
        double shear_v,
        int support,
        int w_support,
        sdp_Mem* facet,
        int facet_offset_l,
        int facet_offset_m,
        sdp_Error* status
);

/* facet(l, m) *= exp(-+2 pi i w_step n w_offset) (inverse: +), complex
 * facets only; nothing for w_offset 0. .h:60-72. */
void sdp_gridder_grid_correct_w_stack(
        int image_size,
        double theta,
        double w_step,
        double shear_u,
        double shear_v,
        sdp_Mem* facet,
        int facet_offset_l,
        int facet_offset_m,
        int w_offset,
        int inverse,
        sdp_Error* status
);

#ifdef __cplusplus
}
#endif

#endif
