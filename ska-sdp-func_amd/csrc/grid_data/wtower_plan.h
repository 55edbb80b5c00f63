// The w-towers plan (sdp_GridderWtowerUVW) as shared by the sub-grid
// gridder (sdp_gridder_wtower_uvw.hip) and the w-stacking driver
// (sdp_grid_wstack_wtower.hip), and the grid-correction arithmetic.
#ifndef SDP_WTOWER_PLAN_H_
#define SDP_WTOWER_PLAN_H_

#include <vector>

#include "ska-sdp-func/grid_data/sdp_gridder_wtower_uvw.h"
#include "wtower_dev.h"
#include "../fft/fft2d.h"

struct sdp_GridderWtowerUVW
{
    int image_size;
    int subgrid_size;
    double theta;
    double w_step;
    double shear_u;
    double shear_v;
    int support;
    int oversampling;
    int w_support;
    int w_oversampling;
    int num_w_planes[2];
    std::vector<double>* uv_kernel;
    std::vector<double>* w_kernel;
    std::vector<double>* w_pattern;       // interleaved complex double
    // Device copies (created on first use).
    double* d_uv_kernel;
    double* d_w_kernel;
    double* d_w_pattern;
    // Grid-correction tables (created on first use).
    double* d_pswf_lm;                    // [image_size]
    double* d_pswf_n;                     // Legendre coefficients
    int n_pswf_n;
    // Per-precision scratch: stack [w_support, S, S], w image, FFT buffer.
    void* d_scratch[2];
    sdp_fft::Plan2D* fft[2];
};

namespace sdp_wt {

// Kernel tables and w-pattern on the device (created once per plan).
void plan_ensure_device(sdp_GridderWtowerUVW* plan, sdp_Error* status);

// PSWF tables of the grid correction on the device.
void plan_ensure_correction(sdp_GridderWtowerUVW* plan, sdp_Error* status);

// Everything the correction of one pixel needs.
struct CorrParams
{
    int image_size;
    double theta, w_step, shear_u, shear_v;
    const double* pswf_lm;    // [image_size]
    const double* pswf_n;     // Legendre coefficients of pswf_n
    int n_pswf_n;
    double c_n;
    int w_offset;
    int inverse;              // grid_correct (1) or degrid_correct (0)
    const double* pn_tab;     // optional [image_size^2] table of pn_value
    // Optional [image_size^2] tables of the whole per-pixel scale
    // 1 / (pswf(l) pswf(m) pswf_n(n)), a geometric constant of the plan:
    // f64 for double facets, f32 (the value the f32 facets multiply by)
    // for float facets. When set, pn_tab is not read.
    const double* scale_f64;
    const float* scale_f32;
};

// 1 / (pswf(l) pswf(m) pswf_n(n)) of pixel (pl, pm) inside the image.
__device__ __forceinline__ double pixel_scale(int pl, int pm,
        const CorrParams& cp);

// pswf_n(|2 w_step n|) of pixel (pl, pm) (1 outside the PSWF's support).
__device__ __forceinline__ double pn_value(int pl, int pm,
        const CorrParams& cp)
{
#pragma clang fp contract(off)
    if (!(cp.c_n > 0.0)) return 1.0;
    const double l = pl * cp.theta / cp.image_size;
    const double m = pm * cp.theta / cp.image_size;
    const double n = lm_to_n_dev(l, m, cp.shear_u, cp.shear_v);
    const double n_x = fabs(n * 2.0 * cp.w_step);
    return (n_x < 1.0) ? pswf_eval(cp.pswf_n, cp.n_pswf_n, n_x) : 1.0;
}

__device__ __forceinline__ double pixel_scale(int pl, int pm,
        const CorrParams& cp)
{
#pragma clang fp contract(off)
    const int half = cp.image_size / 2;
    const double p_l = cp.pswf_lm[pl + half];
    const double p_m = cp.pswf_lm[pm + half];
    const double p_n = cp.pn_tab ?
            cp.pn_tab[(int64_t)(pl + half) * cp.image_size + (pm + half)] :
            pn_value(pl, pm, cp);
    return 1.0 / (p_l * p_m * p_n);
}

CorrParams corr_params(const sdp_GridderWtowerUVW* plan, int w_offset,
        bool inverse);

// Pixel (pl, pm) relative to the image centre inside the facet.
__device__ __forceinline__ bool corr_inside(int pl, int pm,
        const CorrParams& cp)
{
    const int half = cp.image_size / 2;
    return pl + half >= 0 && pl + half < cp.image_size && pm + half >= 0 &&
            pm + half < cp.image_size;
}

// The pixel's 1 / (pswf(l) pswf(m) pswf_n(n)): from the plan's table when
// there is one for the facet's precision, else evaluated.
__device__ __forceinline__ double corr_scale(int pl, int pm, int kind,
        const CorrParams& cp)
{
    const int half = cp.image_size / 2;
    const int64_t idx = (int64_t)(pl + half) * cp.image_size + (pm + half);
    return cp.scale_f64 ? cp.scale_f64[idx] :
            (cp.scale_f32 && (kind == 0 || kind == 2)) ?
            (double)cp.scale_f32[idx] : pixel_scale(pl, pm, cp);
}

// correct_value with the pixel's scale already looked up (callers batch
// the table loads of several pixels ahead of the arithmetic).
__device__ __forceinline__ Cx<double> correct_scaled(Cx<double> z, int kind,
        int pl, int pm, const CorrParams& cp, double scale)
{
#pragma clang fp contract(off)
    if (kind <= 1)
    {
        z.re *= (kind == 0) ? (double)(float)scale : scale;
        return z;
    }
    if (kind == 2)
    {
        const float s = (float)scale;
        z.re = (double)((float)z.re * s);
        z.im = (double)((float)z.im * s);
    }
    else
    {
        z.re *= scale;
        z.im *= scale;
    }
    if (cp.w_offset != 0)
    {
        const double l = pl * cp.theta / cp.image_size;
        const double m = pm * cp.theta / cp.image_size;
        const double n = lm_to_n_dev(l, m, cp.shear_u, cp.shear_v);
        // exp(2 pi i w_step n w_offset): the phase in turns is reduced to
        // [-1/2, 1/2] in double before the (short-argument) sincospi.
        const double turns = cp.w_step * n * cp.w_offset;
        double sn, cs;
        sincospi(2.0 * (turns - rint(turns)), &sn, &cs);
        Cx<double> w = cx<double>(cs, sn);
        if (!cp.inverse) w = cdiv(cx<double>(1.0, 0.0), w);
        if (kind == 2)
        {
            const float wr = (float)w.re, wi = (float)w.im;
            const float zr = (float)z.re, zi = (float)z.im;
            z.re = zr * wr - zi * wi;
            z.im = zr * wi + zi * wr;
        }
        else
        {
            z = cmul(z, w);
        }
    }
    return z;
}

// correct_scaled for a complex-float grid (kind 2) in the image-side passes
// of the w-stack imager (k_image_update, k_image_to_grid, the fused column
// pass of es_fft_wstack.h): the same f32 scale and f32 complex product; the
// w-stack phase w_step n w_offset is formed and reduced to [-1/2, 1/2]
// turns in double as there, but its sine and cosine are taken in single
// precision (sincospif of the reduced phase, ~1 ulp of the f32 values
// correct_scaled rounds its double ones to) instead of double sincospi:
// the double trigonometry was most of those passes' time at config 4
// (1.9 ms per 16384^2 plane).
__device__ __forceinline__ Cx<double> correct_scaled_f32(Cx<double> z, int pl,
        int pm, const CorrParams& cp, float scale)
{
#pragma clang fp contract(off)
    float zr = (float)z.re * scale;
    float zi = (float)z.im * scale;
    if (cp.w_offset != 0)
    {
        // Pixel size and w_step w_offset as one factor each (no double
        // division per pixel; the phase moves by ~1 ulp of a double).
        const double px = cp.theta / cp.image_size;
        const double l = pl * px;
        const double m = pm * px;
        const double n = lm_to_n_dev(l, m, cp.shear_u, cp.shear_v);
        const double turns = (cp.w_step * cp.w_offset) * n;
        float sn, cs;
        sincospif(2.0f * (float)(turns - rint(turns)), &sn, &cs);
        // |w| = 1: 1 / w = conj(w) (degrid_correct).
        const float wr = cs, wi = cp.inverse ? sn : -sn;
        const float xr = zr * wr - zi * wi;
        const float xi = zr * wi + zi * wr;
        zr = xr;
        zi = xi;
    }
    return cx<double>(zr, zi);
}

// Pixel (pl, pm) relative to the image centre of a facet of element kind
// `kind` (AnyView): 1 / (pswf(l) pswf(m) pswf_n(n)), then, for complex
// facets, the w-stacking phasor exp(+-2 pi i w_step n w_offset)
// (sdp_gridder_grid_correct.cpp:18-116), in the facet's precision.
// Pixels outside the image (undefined in the reference) are unchanged.
__device__ __forceinline__ Cx<double> correct_value(Cx<double> z, int kind,
        int pl, int pm, const CorrParams& cp)
{
    if (!corr_inside(pl, pm, cp)) return z;
    return correct_scaled(z, kind, pl, pm, cp, corr_scale(pl, pm, kind, cp));
}

} // namespace sdp_wt

#endif
