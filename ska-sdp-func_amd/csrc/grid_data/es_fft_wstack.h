// Fused image side of the w-stacking imager (sdp_grid_wstack_wtower.hip) on
// the FFT machinery of es_fft.hip: a w-stack plane's inverse FFT with the
// corrected image update in its last column pass (ref
// sdp_grid_wstack_wtower.cpp:686-711).
#ifndef SDP_ES_FFT_WSTACK_H_
#define SDP_ES_FFT_WSTACK_H_

#include "es_fft.h"
#include "wtower_plan.h"

namespace sdp_es {

// image (G x G, any AnyView kind) += grid_correct(checker(IFFT2(grid)) *
// norm) for a w-stack plane (cp: its correction, w_offset included); the
// grid buffer is used as scratch (in place). G a power of two in [1024,
// 16384] with tw its twiddles.
int fft2d_wstack_grid_image(float* grid, int grid_size, const FftTwiddles& tw,
        const sdp_wt::AnyView& image, float norm,
        const sdp_wt::CorrParams& cp, hipStream_t stream);

} // namespace sdp_es

#endif
