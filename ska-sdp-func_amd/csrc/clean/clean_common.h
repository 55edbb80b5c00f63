// Device pieces shared by the CLEAN kernels (Hogbom and multi-scale):
// first-maximum reductions and the Gaussian CLEAN beam.
#ifndef SDP_CLEAN_COMMON_H_
#define SDP_CLEAN_COMMON_H_

#include <climits>
#include <cmath>

#include <hip/hip_runtime.h>

namespace sdp_clean {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

struct Peak
{
    double v;
    long long i;
};

// Larger value wins; ties go to the lower flat index (first maximum).
__device__ __forceinline__ bool better(double v, long long i, double bv,
        long long bi)
{
    return v > bv || (v == bv && i < bi);
}

__device__ __forceinline__ void wave_best(double& v, long long& i)
{
    for (int o = 32; o > 0; o >>= 1)
    {
        const double ov = __shfl_xor(v, o, 64);
        const long long oi = __shfl_xor(i, o, 64);
        if (better(ov, oi, v, i))
        {
            v = ov;
            i = oi;
        }
    }
}

// Workgroup-wide best (value, index); result valid in thread 0. Contains a
// barrier: every thread of the workgroup must call it.
__device__ __forceinline__ void block_best(double& v, long long& i)
{
    __shared__ double s_v[kWaves];
    __shared__ long long s_i[kWaves];
    wave_best(v, i);
    const int w = threadIdx.x >> 6;
    __syncthreads();             // previous use of s_v / s_i complete
    if ((threadIdx.x & 63) == 0)
    {
        s_v[w] = v;
        s_i[w] = i;
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
        for (int k = 1; k < kWaves; ++k)
        {
            if (better(s_v[k], s_i[k], v, i))
            {
                v = s_v[k];
                i = s_i[k];
            }
        }
    }
}

// Gaussian CLEAN beam value at (x, y) of an nb x nb table centred on
// (nb / 2, nb / 2) (sdp_hogbom_clean.cpp:33-80, sdp_ms_clean_cornwell.cpp
// :31-78), in double.
__device__ __forceinline__ double cbeam_value(int x, int y, int nb,
        double sx, double sy, double theta_deg)
{
    const double th = (M_PI / 180) * theta_deg;
    const double ct = cos(th), st = sin(th), s2 = sin(2 * th);
    const double a = ct * ct / (2 * sx * sx) + st * st / (2 * sy * sy);
    const double b = s2 / (4 * sx * sx) - s2 / (4 * sy * sy);
    const double c = st * st / (2 * sx * sx) + ct * ct / (2 * sy * sy);
    const int c0 = nb / 2;
    const double dx = x - c0, dy = y - c0;
    return exp(-(a * dx * dx + 2 * b * dx * dy + c * dy * dy));
}

} // namespace sdp_clean

#endif
