// 2-D complex-to-complex FFT on MI355X via rocFFT (in place, unnormalised).
// Replaces the cuFFT plan of the reference's sdp_fft (sdp_fft.cpp:362-448,
// 883-921): same convention (inverse = +i exponent, no scaling). Plans are
// created once per gridder plan instead of once per call.
#ifndef SDP_FFT2D_H_
#define SDP_FFT2D_H_

#include <hip/hip_runtime.h>

#include "ska-sdp-func/utility/sdp_errors.h"

namespace sdp_fft {

struct Plan2D;

// n_slow x n_fast row-major complex array; dbl selects complex128.
Plan2D* create_2d(int n_slow, int n_fast, bool dbl, sdp_Error* status);
// `batch` n_slow x n_fast arrays, `distance` elements apart (in place).
Plan2D* create_2d_batched(int n_slow, int n_fast, bool dbl, size_t batch,
        size_t distance, sdp_Error* status);
void exec_2d(Plan2D* plan, void* data, bool forward, hipStream_t stream,
        sdp_Error* status);
void destroy_2d(Plan2D* plan);

} // namespace sdp_fft

#endif
