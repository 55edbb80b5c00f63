// Image-plane device helpers shared by the image kernels (es_kernels.hip)
// and the fused FFT passes (es_fft.hip): the w-correction quadrature, the
// separable 1/correction and the w-screen phasor, in working precision T.
#ifndef SDP_ES_IMAGE_DEV_H_
#define SDP_ES_IMAGE_DEV_H_

#include <cmath>
#include <cstdint>
#include <type_traits>

#include <hip/hip_runtime.h>

#include "es_kernels.h"

namespace sdp_es {
namespace img {

constexpr double kPi = 3.1415926535897931;

// conv_corr device function, kernels.cu:69-87 (cos argument in double as the
// reference's double PI literal promotes it).
template<typename T>
__device__ __forceinline__ T conv_corr_n(const ImageParams<T>& ip, T k)
{
    const T support = (T)ip.support;
    const uint32_t np = (uint32_t)ceil(T(1.5) * support + T(2));
    T c = T(0);
    for (uint32_t i = 0; i < np; ++i)
    {
        // The argument in double as the reference forms it; in a float
        // plan it is reduced to [-pi, pi] in double first and its cosine
        // taken in float (the term is rounded to float anyway): the
        // argument reaches tens of radians, and rounding it to float
        // unreduced would cost ~|arg| * 6e-8 absolute per term; reduced,
        // the error stays within ~2e-7 absolute, at a fraction of the FP64
        // libm cost (14 terms per pixel of the 3-D correction).
        const double arg = kPi * (double)k * (double)support *
                (double)ip.quad_nodes[i];
        double cs;
        if (std::is_same<T, float>::value)
        {
            const double red = arg - (2.0 * kPi) *
                    rint(arg * (0.5 / kPi));
            cs = (double)cosf((float)red);
        }
        else
        {
            cs = cos(arg);
        }
        c = (T)((double)c + (double)ip.quad_kernel[i] * cs *
                (double)ip.quad_weights[i]);
    }
    return c * support;
}

// 1 / correction at pixel offsets (i = |x| column, j = |y| row),
// kernels.cu:711-740.
template<typename T>
__device__ __forceinline__ T inv_correction(const ImageParams<T>& ip, int i, int j)
{
#pragma clang fp contract(off)
    const T l_conv = ip.conv_corr[i], m_conv = ip.conv_corr[j];
    T corr;
    if (ip.do_w)
    {
        const T l = ip.pixel_size * (T)i, m = ip.pixel_size * (T)j;
        const T n = sqrt(T(1) - l * l - m * m) - T(1);
        T n_conv = conv_corr_n(ip, n * ip.inv_w_scale);
        n_conv *= (ip.norm * ip.norm);
        corr = l_conv * m_conv * n_conv;
    }
    else
    {
        corr = l_conv * m_conv * ip.norm * ip.norm;
    }
    return T(1) / corr;
}

__device__ __forceinline__ void sin_cos(float x, float* s, float* c)
{
    sincosf(x, s, c);
}
__device__ __forceinline__ void sin_cos(double x, double* s, double* c)
{
    sincos(x, s, c);
}

// w-screen phasor, kernels.cu:110-123.
template<typename T>
__device__ __forceinline__ void phasor(const ImageParams<T>& ip, int plane, int i, int j,
        T sign, T& re, T& im)
{
#pragma clang fp contract(off)
    const T l = ip.pixel_size * (T)i, m = ip.pixel_size * (T)j;
    const T w = (T)plane * ip.inv_w_scale + ip.min_plane_w;
    const T sos = l * l + m * m;
    const T nm1 = (-sos) / (sqrt(T(1) - sos) + T(1));
    const T x = T(2) * T(kPi) * w * nm1;
    const T xn = T(1) / (nm1 + T(1));
    sin_cos(sign * x, &im, &re);
    re *= xn;
    im *= xn;
}

} // namespace img
} // namespace sdp_es

#endif
