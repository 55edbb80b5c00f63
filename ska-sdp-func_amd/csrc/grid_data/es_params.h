// Host-side parameter maths of the ES-FFT gridder.
// Follows src/ska-sdp-func/grid_data/sdp_gridder_uvw_es_fft_utils.cpp of the
// reference (kernel-table lookup :225-537, Gauss-Legendre correction tables
// :13-175, good_size :181-218); pinned by tests/golden/es_params.json.
#ifndef SDP_ES_PARAMS_H_
#define SDP_ES_PARAMS_H_

#include "ska-sdp-func/utility/sdp_errors.h"

namespace sdp_es {

constexpr int kQuadratureBound = 32;   // QUADRATURE_SUPPORT_BOUND

int good_size_complex(int n);

// Grid size, support and beta/support for accuracy epsilon.
void params_from_epsilon(double epsilon, int image_size, bool is_double,
        int* grid_size, int* support, double* beta_over_support);

// beta is the FULL beta (table value * support). conv_corr has
// image_size/2 + 1 entries; the quadrature arrays kQuadratureBound entries.
// Returns the normalisation factor C(0).
double gauss_legendre_conv_kernel(int image_size, int grid_size, int support,
        double beta, double* quad_kernel, double* quad_nodes,
        double* quad_weights, double* conv_corr);

} // namespace sdp_es

#endif
