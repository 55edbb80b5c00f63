// Host-side kernel math of the w-towers gridder (double precision).
//
// The reference evaluates the prolate spheroidal angular function S_00(c, x)
// with a port of Zhang & Jin's specfun routines (sdp_pswf.cpp,
// private_pswf.h). Here it is computed independently: S_00 is the ground
// state of the Sturm-Liouville operator -d/dx (1 - x^2) d/dx + c^2 x^2,
// which is a symmetric tridiagonal matrix in the orthonormal even Legendre
// basis; its lowest eigenvector (Sturm bisection + inverse iteration) gives
// the Legendre coefficients, normalised to S(0) = 1 (Flammer's convention,
// the one specfun uses). Agreement with specfun (scipy.special.pro_ang1) is
// checked in tests/test_wtower_oracle.py.
#ifndef SDP_WTOWER_MATH_H_
#define SDP_WTOWER_MATH_H_

#include <cmath>
#include <complex>
#include <vector>

namespace sdp_wt {

struct Pswf
{
    double c = 0.0;
    int m = 0;                  // order (n = m)
    // m = 0: coefficients of P_0, P_2, P_4, ...; m > 0: of the associated
    // Legendre functions P_m^m, P_{m+2}^m, ... (no Condon-Shortley phase).
    std::vector<double> coef;
    double operator()(double x) const;
};

Pswf make_pswf(double c);

// S_mm(c, x) of order m >= 0 in Flammer's normalisation
// (S_mm(c, 0) = P_m^m(0) = (2m - 1)!!), the function the reference's
// sdp_pswf_create(m, c) evaluates (sdp_pswf.cpp:612-635). m = 0 is
// make_pswf(c).
Pswf make_pswf_order(double c, int m);

// sdp_pswf.cpp:570-601: values on `size` points x = 2 i / size about the
// centre; out[0] = 0 (1e-15 with end_correction and even size).
std::vector<double> generate_pswf(double c, int size, bool end_correction);

// sdp_gridder_utils.cpp:385-427: oversampled kernel
// [(oversampling + 1) x support] from an image-space window of `support`.
std::vector<double> make_kernel(const std::vector<double>& window,
        int oversampling);

// sdp_gridder_utils.cpp:1329-1350.
std::vector<double> make_pswf_kernel(int support, int oversampling);

// sdp_gridder_utils.h:399-412.
inline double lm_to_n(double l, double m, double h_u, double h_v)
{
    if (h_u == 0 && h_v == 0) return std::sqrt(1 - l * l - m * m) - 1;
    const double a = h_u * l + h_v * m - 1;
    const double b = h_u * h_u + h_v * h_v + 1;
    return (std::sqrt(a * a - b * (l * l + m * m)) + a) / b;
}

// sdp_gridder_utils.cpp:1353-1380, [subgrid_size x subgrid_size].
std::vector<std::complex<double> > make_w_pattern(int subgrid_size,
        double theta, double shear_u, double shear_v, double w_step);

// sdp_gridder_utils.cpp:1016-1039.
double determine_w_step(double theta, double fov, double shear_u,
        double shear_v, double x0);

} // namespace sdp_wt

#endif
