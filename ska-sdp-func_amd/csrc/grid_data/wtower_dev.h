// Device-side pieces of the w-towers gridder shared by its kernels:
// complex arithmetic in the precision of each step, typed array views,
// the channel clamp and the Legendre-series PSWF evaluation.
#ifndef SDP_WTOWER_DEV_H_
#define SDP_WTOWER_DEV_H_

#include <cstdint>

#include <hip/hip_runtime.h>

#include "ska-sdp-func/utility/sdp_mem.h"

namespace sdp_wt {

constexpr double kC0 = 299792458.0;

template<typename T>
struct Cx
{
    T re, im;
};

template<typename T>
__device__ __forceinline__ Cx<T> cx(T re, T im)
{
    Cx<T> z;
    z.re = re;
    z.im = im;
    return z;
}

template<typename T>
__device__ __forceinline__ Cx<T> cmul(Cx<T> a, Cx<T> b)
{
#pragma clang fp contract(off)
    return cx<T>(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re);
}

// a / b for complex double with Smith's scaling, as libgcc's __divdc3
// (which the reference's std::complex division calls) for finite operands
// of ordinary magnitude.
__device__ __forceinline__ Cx<double> cdiv(Cx<double> a, Cx<double> b)
{
#pragma clang fp contract(off)
    if (fabs(b.re) < fabs(b.im))
    {
        const double ratio = b.re / b.im;
        const double denom = b.re * ratio + b.im;
        return cx<double>((a.re * ratio + a.im) / denom,
                (a.im * ratio - a.re) / denom);
    }
    const double ratio = b.im / b.re;
    const double denom = b.im * ratio + b.re;
    return cx<double>((a.im * ratio + a.re) / denom,
            (a.im - a.re * ratio) / denom);
}

// z ** n as libstdc++'s pow(complex, int): binary exponentiation of |n|,
// reciprocal for n < 0.
__device__ __forceinline__ Cx<double> cpow_int(Cx<double> z, int n)
{
#pragma clang fp contract(off)
    unsigned k = (n < 0) ? (unsigned)(-n) : (unsigned)n;
    Cx<double> y = (k % 2) ? z : cx<double>(1.0, 0.0);
    while (k >>= 1)
    {
        z = cmul(z, z);
        if (k % 2) y = cmul(y, z);
    }
    return (n < 0) ? cdiv(cx<double>(1.0, 0.0), y) : y;
}

// Any of f32 / f64 / c64 / c128, read and written as complex double.
struct AnyView
{
    void* ptr;
    int kind;   // 0 f32, 1 f64, 2 c64, 3 c128

    __device__ __forceinline__ Cx<double> load(int64_t i) const
    {
        switch (kind)
        {
        case 0: return cx<double>(((const float*)ptr)[i], 0.0);
        case 1: return cx<double>(((const double*)ptr)[i], 0.0);
        case 2:
            return cx<double>(((const float*)ptr)[2 * i],
                    ((const float*)ptr)[2 * i + 1]);
        default:
            return cx<double>(((const double*)ptr)[2 * i],
                    ((const double*)ptr)[2 * i + 1]);
        }
    }

    __device__ __forceinline__ void store(int64_t i, Cx<double> z) const
    {
        switch (kind)
        {
        case 0: ((float*)ptr)[i] = (float)z.re; break;
        case 1: ((double*)ptr)[i] = z.re; break;
        case 2:
            ((float*)ptr)[2 * i] = (float)z.re;
            ((float*)ptr)[2 * i + 1] = (float)z.im;
            break;
        default:
            ((double*)ptr)[2 * i] = z.re;
            ((double*)ptr)[2 * i + 1] = z.im;
        }
    }
};

inline int any_kind(sdp_MemType t)
{
    switch (t)
    {
    case SDP_MEM_FLOAT: return 0;
    case SDP_MEM_DOUBLE: return 1;
    case SDP_MEM_COMPLEX_FLOAT: return 2;
    case SDP_MEM_COMPLEX_DOUBLE: return 3;
    default: return -1;
    }
}

// sdp_gridder_clamp_channels.h:86-146 (the inline form used by the
// sub-grid kernels).
__device__ __forceinline__ void clamp_inline(double u, double freq0_hz,
        double dfreq_hz, int64_t* start_ch, int64_t* end_ch, double min_u,
        double max_u)
{
#pragma clang fp contract(off)
    const double u0 = freq0_hz * u / kC0;
    const double du = dfreq_hz * u / kC0;
    const double min_u_rel = fabs(min_u - u0);
    const double max_u_rel = fabs(max_u - u0);
    const double eta = fmax(min_u_rel, max_u_rel) / 2147483645.0;
    if (du > eta)
    {
        const int64_t s = (int64_t)ceil((min_u - u0) / du);
        const int64_t e = (int64_t)ceil((max_u - u0) / du);
        *start_ch = *start_ch > s ? *start_ch : s;
        *end_ch = *end_ch < e ? *end_ch : e;
    }
    else if (du < -eta)
    {
        const int64_t s = (int64_t)ceil((max_u - u0) / du);
        const int64_t e = (int64_t)ceil((min_u - u0) / du);
        *start_ch = *start_ch > s ? *start_ch : s;
        *end_ch = *end_ch < e ? *end_ch : e;
    }
    else
    {
        if (min_u > u0 || max_u <= u0)
        {
            *start_ch = 0;
            *end_ch = 0;
        }
    }
    if (*end_ch <= *start_ch)
    {
        *start_ch = 0;
        *end_ch = 0;
    }
}

// S_00(c, x) = sum_k coef[k] P_2k(x) (see wtower_math.h).
__device__ __forceinline__ double pswf_eval(const double* coef, int n,
        double x)
{
    double p_prev = 1.0, p_cur = x, sum = coef[0];
    const int nmax = 2 * (n - 1);
    for (int deg = 1; deg < nmax; ++deg)
    {
        const double p_next = ((2.0 * deg + 1) * x * p_cur - deg * p_prev) /
                (deg + 1);
        p_prev = p_cur;
        p_cur = p_next;
        if ((deg + 1) % 2 == 0) sum += coef[(deg + 1) / 2] * p_cur;
    }
    return sum;
}

__device__ __forceinline__ double lm_to_n_dev(double l, double m, double h_u,
        double h_v)
{
#pragma clang fp contract(off)
    if (h_u == 0 && h_v == 0) return sqrt(1 - l * l - m * m) - 1;
    const double a = h_u * l + h_v * m - 1;
    const double b = h_u * h_u + h_v * h_v + 1;
    return (sqrt(a * a - b * (l * l + m * m)) + a) / b;
}

// floor(x / d) for d > 0 and |x| < 2^24: a float estimate, corrected once.
__device__ __forceinline__ int floor_div_small(int x, int d, float inv_d)
{
    int q = (int)floorf((float)x * inv_d);
    const int r = x - q * d;
    if (r < 0) --q;
    else if (r >= d) ++q;
    return q;
}

// Sub-grids along one axis that cover grid cell x0 (relative to the first
// sub-grid origin, G/2 - S/2 cells from the grid's first cell), in the
// reference's task order (wrap k = -1, 0, 1, then index; utils.cpp:553-601):
// off[] the cell's offset inside each, idx[] its sub-grid index minus
// lo_idx; returns how many (at most NC, host-checked).
template<int NC>
__device__ __forceinline__ int gather_candidates(int x0, int G, int S,
        int eff, float inv_eff, int lo_idx, int n_idx, int (&off)[NC],
        int (&idx)[NC])
{
    int nc = 0;
    for (int k = -1; k <= 1; ++k)
    {
        const int x = x0 + k * G;
        const int i_lo = max(floor_div_small(x - S + eff, eff, inv_eff),
                lo_idx);
        const int i_hi = min(floor_div_small(x, eff, inv_eff),
                lo_idx + n_idx - 1);
        for (int ii = i_lo; ii <= i_hi; ++ii)
        {
            const int o = x - ii * eff;
            if (o < 0 || o >= S || nc >= NC) continue;
            off[nc] = o;
            idx[nc] = ii - lo_idx;
            ++nc;
        }
    }
    return nc;
}

} // namespace sdp_wt

#endif
