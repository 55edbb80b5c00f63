// MI355X-native w-towers sub-grid (de)gridder.
//
// Replaces src/ska-sdp-func/grid_data/sdp_gridder_wtower_uvw.cpp/.cu of
// ska-sdp-func 1.2.2 (see the header for the ABI). Per call:
//   - the w range of the selected visibilities (device reduction) gives the
//     w-planes to visit (.cpp:784-792, 991-999);
//   - a stack of w_support sub-grid layers is moved through the planes: one
//     S x S FFT (rocFFT) per plane plus w-pattern multiplications; the stack
//     is a ring buffer (the reference copies it down one layer per plane);
//   - per plane, one HIP kernel (de)grids every row with the oversampled
//     PSWF kernels (w_support x support x support taps per visibility), in
//     the reference's loop order and precision; gridding adds with device
//     atomics (as the reference GPU kernel).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ska-sdp-func/grid_data/sdp_gridder_wtower_uvw.h"
#include "wtower_dev.h"
#include "wtower_math.h"
#include "wtower_ops.h"
#include "wtower_plan.h"
#include "../fft/fft2d.h"
#include "../utility/sdp_hip.h"

using namespace sdp_wt;


namespace {

struct WtParams
{
    int S, support, w_support, os, wos;
    double theta, w_step;
    int off_u, off_v, off_w;
    double f0, df;
    int64_t start_row, end_row;
    int w_plane;
    int ring;          // stack layer of iw = 0
    int64_t num_chan;
};

// Row selection and per-channel kernel offsets (.cpp:80-140 / 387-438).
struct RowSel
{
    int64_t s, e;
    double uvw0[3], duvw[3];
};

template<typename U>
__device__ __forceinline__ bool select_row(const WtParams& p,
        const U* __restrict__ uvws, const int* __restrict__ start_chs,
        const int* __restrict__ end_chs, int64_t r, RowSel& sel)
{
#pragma clang fp contract(off)
    sel.s = start_chs[r];
    sel.e = end_chs[r];
    if (sel.s >= sel.e) return false;
    // Channel ranges beyond the vis array are undefined in the reference;
    // keep every access inside it.
    sel.s = sel.s < 0 ? 0 : sel.s;
    sel.e = sel.e > p.num_chan ? p.num_chan : sel.e;
    if (sel.s >= sel.e) return false;
    const U uvw[3] = {uvws[3 * r], uvws[3 * r + 1], uvws[3 * r + 2]};
    const double min_w = (p.w_plane + p.off_w - 1) * p.w_step;
    const double max_w = (p.w_plane + p.off_w) * p.w_step;
    clamp_inline((double)uvw[2], p.f0, p.df, &sel.s, &sel.e, min_w, max_w);
    if (sel.s >= sel.e) return false;
    const double s_uvw0 = p.f0 / kC0, s_duvw = p.df / kC0;
    for (int k = 0; k < 3; ++k)
    {
        sel.uvw0[k] = uvw[k] * s_uvw0;
        sel.duvw[k] = uvw[k] * s_duvw;
    }
    sel.uvw0[0] -= p.off_u / p.theta;
    sel.uvw0[1] -= p.off_v / p.theta;
    sel.uvw0[2] -= ((p.off_w + p.w_plane - 1) * p.w_step);
    const int half = p.S / 2;
    const double u_min = floor(p.theta * (sel.uvw0[0] + sel.s * sel.duvw[0]));
    const double u_max = ceil(p.theta * (sel.uvw0[0] + (sel.e - 1) * sel.duvw[0]));
    const double v_min = floor(p.theta * (sel.uvw0[1] + sel.s * sel.duvw[1]));
    const double v_max = ceil(p.theta * (sel.uvw0[1] + (sel.e - 1) * sel.duvw[1]));
    return !(u_min < -half || u_max >= half || v_min < -half || v_max >= half);
}

struct Taps
{
    int iu0, iv0, u_off, v_off, w_off;
    bool valid;   // false: negative oversampled index (kernel tables would
                  // be read before their start -- undefined in the
                  // reference); the visibility is skipped
};

__device__ __forceinline__ Taps taps_for(const WtParams& p, const RowSel& sel,
        int64_t c)
{
#pragma clang fp contract(off)
    const double u = sel.uvw0[0] + c * sel.duvw[0];
    const double v = sel.uvw0[1] + c * sel.duvw[1];
    const double w = sel.uvw0[2] + c * sel.duvw[2];
    const double theta_ov = p.theta * p.os;
    const double w_step_ov = 1.0 / p.w_step * p.wos;
    const int half_ov = (p.S / 2 - p.support / 2 + 1) * p.os;
    const int iu0_ov = int(round(u * theta_ov)) + half_ov;
    const int iv0_ov = int(round(v * theta_ov)) + half_ov;
    const int iw0_ov = int(round(w * w_step_ov));
    Taps t;
    t.iu0 = iu0_ov / p.os;
    t.iv0 = iv0_ov / p.os;
    t.u_off = (iu0_ov % p.os) * p.support;
    t.v_off = (iv0_ov % p.os) * p.support;
    t.w_off = (iw0_ov % p.wos) * p.w_support;
    t.valid = iu0_ov >= 0 && iv0_ov >= 0 && iw0_ov >= 0;
    return t;
}

// Offset of stack cell (iw, iu, iv) of the reference's contiguous
// [w_support, S, S] stack, through the ring of layers. Taps within a layer
// take the fast path; taps outside one (possible only when visibilities
// come within support / 2 of the sub-grid edge) wrap into the neighbouring
// layer exactly as the reference's flat indexing does, and taps outside
// the whole stack -- undefined in the reference -- are dropped (-1).
__device__ __forceinline__ int64_t stack_cell(const WtParams& p, int iw,
        int iu, int iv)
{
    const int64_t layer = (int64_t)p.S * p.S;
    const int64_t f = ((int64_t)iw * p.S + iu) * p.S + iv;
    if (f < 0 || f >= p.w_support * layer) return -1;
    const int l = (int)(f / layer);
    return ((p.ring + l) % p.w_support) * layer + (f - l * layer);
}

__device__ __forceinline__ bool taps_inside(const WtParams& p, const Taps& t)
{
    return t.iu0 >= 0 && t.iu0 + p.support <= p.S && t.iv0 >= 0 &&
            t.iv0 + p.support <= p.S;
}

// One visibility from the stack (.cpp:143-171), in the vis precision.
template<typename T, bool INSIDE>
__device__ __forceinline__ Cx<T> degrid_one(const WtParams& p,
        const Taps& t, const Cx<T>* __restrict__ stack,
        const double* __restrict__ uv_kernel,
        const double* __restrict__ w_kernel)
{
#pragma clang fp contract(off)
    const int64_t layer = (int64_t)p.S * p.S;
    Cx<T> local = cx<T>(0, 0);
    for (int iw = 0; iw < p.w_support; ++iw)
    {
        const Cx<T>* sub = stack + ((p.ring + iw) % p.w_support) * layer;
        Cx<T> lu = cx<T>(0, 0);
        for (int iu = 0; iu < p.support; ++iu)
        {
            const Cx<T>* row = sub + (int64_t)(t.iu0 + iu) * p.S + t.iv0;
            Cx<T> lv = cx<T>(0, 0);
            for (int iv = 0; iv < p.support; ++iv)
            {
                Cx<T> g;
                if (INSIDE)
                {
                    g = row[iv];
                }
                else
                {
                    const int64_t i = stack_cell(p, iw, t.iu0 + iu,
                            t.iv0 + iv);
                    g = (i < 0) ? cx<T>(0, 0) : stack[i];
                }
                const T k = (T)uv_kernel[t.v_off + iv];
                lv.re += k * g.re;
                lv.im += k * g.im;
            }
            const T k = (T)uv_kernel[t.u_off + iu];
            lu.re += k * lv.re;
            lu.im += k * lv.im;
        }
        const T k = (T)w_kernel[t.w_off + iw];
        local.re += k * lu.re;
        local.im += k * lu.im;
    }
    return local;
}

// Thread per row: each selected channel of the row is degridded from the
// stack and added to vis (.cpp:45-176).
template<typename T, typename U>
__global__ void k_wt_degrid(WtParams p, const Cx<T>* __restrict__ stack,
        const U* __restrict__ uvws, const int* __restrict__ start_chs,
        const int* __restrict__ end_chs, const double* __restrict__ uv_kernel,
        const double* __restrict__ w_kernel, Cx<T>* __restrict__ vis)
{
#pragma clang fp contract(off)
    const int64_t r = p.start_row + blockIdx.x * (int64_t)blockDim.x +
            threadIdx.x;
    if (r >= p.end_row) return;
    RowSel sel;
    if (!select_row(p, uvws, start_chs, end_chs, r, sel)) return;
    for (int64_t c = sel.s; c < sel.e; ++c)
    {
        const Taps t = taps_for(p, sel, c);
        if (!t.valid) continue;
        const Cx<T> local = taps_inside(p, t) ?
                degrid_one<T, true>(p, t, stack, uv_kernel, w_kernel) :
                degrid_one<T, false>(p, t, stack, uv_kernel, w_kernel);
        Cx<T>& out = vis[r * p.num_chan + c];
        out.re += local.re;
        out.im += local.im;
    }
}

// One visibility onto the stack (.cpp:455-480), device atomics.
template<typename T, bool INSIDE>
__device__ __forceinline__ void grid_one(const WtParams& p, const Taps& t,
        const Cx<T> v, Cx<T>* __restrict__ stack,
        const double* __restrict__ uv_kernel,
        const double* __restrict__ w_kernel)
{
#pragma clang fp contract(off)
    const int64_t layer = (int64_t)p.S * p.S;
    for (int iw = 0; iw < p.w_support; ++iw)
    {
        Cx<T>* sub = stack + ((p.ring + iw) % p.w_support) * layer;
        const T kw = (T)w_kernel[t.w_off + iw];
        const Cx<T> vw = cx<T>(kw * v.re, kw * v.im);
        for (int iu = 0; iu < p.support; ++iu)
        {
            const T ku = (T)uv_kernel[t.u_off + iu];
            const Cx<T> vu = cx<T>(ku * vw.re, ku * vw.im);
            Cx<T>* row = sub + (int64_t)(t.iu0 + iu) * p.S + t.iv0;
            for (int iv = 0; iv < p.support; ++iv)
            {
                Cx<T>* cell;
                if (INSIDE)
                {
                    cell = row + iv;
                }
                else
                {
                    const int64_t i = stack_cell(p, iw, t.iu0 + iu,
                            t.iv0 + iv);
                    if (i < 0) continue;
                    cell = stack + i;
                }
                const T kv = (T)uv_kernel[t.v_off + iv];
                unsafeAtomicAdd(&cell->re, kv * vu.re);
                unsafeAtomicAdd(&cell->im, kv * vu.im);
            }
        }
    }
}

template<typename T, typename U>
__global__ void k_wt_grid(WtParams p, Cx<T>* __restrict__ stack,
        const U* __restrict__ uvws, const int* __restrict__ start_chs,
        const int* __restrict__ end_chs, const double* __restrict__ uv_kernel,
        const double* __restrict__ w_kernel, const Cx<T>* __restrict__ vis)
{
#pragma clang fp contract(off)
    const int64_t r = p.start_row + blockIdx.x * (int64_t)blockDim.x +
            threadIdx.x;
    if (r >= p.end_row) return;
    RowSel sel;
    if (!select_row(p, uvws, start_chs, end_chs, r, sel)) return;
    for (int64_t c = sel.s; c < sel.e; ++c)
    {
        const Taps t = taps_for(p, sel, c);
        if (!t.valid) continue;
        const Cx<T> v = vis[r * p.num_chan + c];
        if (taps_inside(p, t))
            grid_one<T, true>(p, t, v, stack, uv_kernel, w_kernel);
        else
            grid_one<T, false>(p, t, v, stack, uv_kernel, w_kernel);
    }
}

// Grid correction of a facet (sdp_gridder_grid_correct.cpp:18-116).
__global__ void k_grid_correct(AnyView facet, int nl, int nm, int off_l,
        int off_m, CorrParams cp)
{
    const int im = blockIdx.x * blockDim.x + threadIdx.x;
    const int il = blockIdx.y;
    if (im >= nm || il >= nl) return;
    const int64_t i = (int64_t)il * nm + im;
    facet.store(i, correct_value(facet.load(i), facet.kind,
            il - nl / 2 + off_l, im - nm / 2 + off_m, cp));
}

void upload(const std::vector<double>& h, double** d, sdp_Error* status)
{
    if (*d || *status) return;
    SDP_HIP_CHECK(hipMalloc((void**)d, h.size() * sizeof(double)), status);
    if (*status) return;
    SDP_HIP_CHECK(hipMemcpy(*d, h.data(), h.size() * sizeof(double),
            hipMemcpyHostToDevice), status);
}

template<typename T>
size_t scratch_bytes(const sdp_GridderWtowerUVW* plan)
{
    const size_t layer = (size_t)plan->subgrid_size * plan->subgrid_size;
    // stack (T complex) | w image (complex double) | FFT buffer (T complex)
    return layer * (plan->w_support + 1) * 2 * sizeof(T) +
            layer * 2 * sizeof(double);
}

template<typename T>
void ensure_scratch(sdp_GridderWtowerUVW* plan, sdp_Error* status)
{
    const int k = sizeof(T) == 8;
    if (*status || plan->d_scratch[k]) return;
    SDP_HIP_CHECK(hipMalloc(&plan->d_scratch[k], scratch_bytes<T>(plan)),
            status);
    if (!*status)
        plan->fft[k] = sdp_fft::create_2d(plan->subgrid_size,
                plan->subgrid_size, k == 1, status);
}

// First / last w-plane of the rows' channels (.cpp:784-792); false when
// no channel is selected (the reference's range is then undefined).
template<typename U>
bool w_range(const sdp_GridderWtowerUVW* plan, const U* uvws, int64_t rows,
        double f0, double df, const int* s, const int* e, int off_w,
        int* first, int* last, sdp_Error* status)
{
    double lo[3], hi[3];
    uvw_bounds_dev<U>(uvws, rows, f0, df, s, e, lo, hi, status);
    if (*status || !(lo[2] <= hi[2])) return false;
    const double eta = 1e-5;
    *first = (int)floor(lo[2] / plan->w_step - eta) - off_w;
    *last = (int)ceil(hi[2] / plan->w_step + eta) - off_w + 1;
    return true;
}

template<typename T>
void fft_shift(sdp_GridderWtowerUVW* plan, T* data, bool forward,
        sdp_Error* status)
{
    const int k = sizeof(T) == 8;
    wt_fft_phase<T>(data, plan->subgrid_size, plan->subgrid_size, status);
    sdp_fft::exec_2d(plan->fft[k], data, forward, 0, status);
    wt_fft_phase<T>(data, plan->subgrid_size, plan->subgrid_size, status);
}

WtParams base_params(const sdp_GridderWtowerUVW* plan, int off_u, int off_v,
        int off_w, double f0, double df, int64_t r0, int64_t r1,
        int64_t num_chan)
{
    WtParams p;
    p.S = plan->subgrid_size;
    p.support = plan->support;
    p.w_support = plan->w_support;
    p.os = plan->oversampling;
    p.wos = plan->w_oversampling;
    p.theta = plan->theta;
    p.w_step = plan->w_step;
    p.off_u = off_u;
    p.off_v = off_v;
    p.off_w = off_w;
    p.f0 = f0;
    p.df = df;
    p.start_row = r0;
    p.end_row = r1;
    p.w_plane = 0;
    p.ring = 0;
    p.num_chan = num_chan;
    return p;
}

template<typename T, typename U>
void degrid_impl(sdp_GridderWtowerUVW* plan, const sdp_Mem* subgrid_image,
        int off_u, int off_v, int off_w, double f0, double df,
        const sdp_Mem* uvws, const sdp_Mem* start_chs, const sdp_Mem* end_chs,
        sdp_Mem* vis, int64_t r0, int64_t r1, sdp_Error* status)
{
    ensure_scratch<T>(plan, status);
    if (*status) return;
    const int k = sizeof(T) == 8;
    const int S = plan->subgrid_size, ws = plan->w_support;
    const int64_t layer = (int64_t)S * S;
    T* stack = (T*)plan->d_scratch[k];
    T* wimg = stack + 2 * layer * ws;                 // vis precision here
    const U* d_uvw = (const U*)sdp_mem_data_const(uvws);
    const int* d_s = (const int*)sdp_mem_data_const(start_chs);
    const int* d_e = (const int*)sdp_mem_data_const(end_chs);
    int first = 0, last = 0;
    if (!w_range<U>(plan, d_uvw, sdp_mem_shape_dim(uvws, 0), f0, df, d_s,
            d_e, off_w, &first, &last, status))
        return;
    const AnyView wv = {wimg, sizeof(T) == 8 ? 3 : 2};
    const AnyView in = {const_cast<void*>(sdp_mem_data_const(subgrid_image)),
            any_kind(sdp_mem_type(subgrid_image))};
    // w_subgrid_image = subgrid_image / w_pattern ** (first - ws / 2)
    wt_scale_inv(wv, in, plan->d_w_pattern, first - ws / 2, layer, status);
    for (int i = 0; i < ws; ++i)
    {
        T* dst = stack + 2 * layer * i;
        SDP_HIP_CHECK(hipMemcpyAsync(dst, wimg, 2 * layer * sizeof(T),
                hipMemcpyDeviceToDevice, 0), status);
        fft_shift<T>(plan, dst, true, status);
        wt_scale_inv(wv, wv, plan->d_w_pattern, 1, layer, status);
    }
    WtParams p = base_params(plan, off_u, off_v, off_w, f0, df, r0, r1,
            sdp_mem_shape_dim(vis, 1));
    const unsigned blocks = (unsigned)((r1 - r0 + 255) / 256);
    int ring = 0;
    for (int w_plane = first; w_plane <= last && !*status; ++w_plane)
    {
        if (w_plane != first)
        {
            // Drop layer 0, the new last layer = FFT(w image).
            T* dst = stack + 2 * layer * ring;
            ring = (ring + 1) % ws;
            SDP_HIP_CHECK(hipMemcpyAsync(dst, wimg, 2 * layer * sizeof(T),
                    hipMemcpyDeviceToDevice, 0), status);
            fft_shift<T>(plan, dst, true, status);
            wt_scale_inv(wv, wv, plan->d_w_pattern, 1, layer, status);
        }
        p.w_plane = w_plane;
        p.ring = ring;
        if (blocks)
        {
            k_wt_degrid<T, U><<<blocks, 256>>>(p, (const Cx<T>*)stack, d_uvw,
                    d_s, d_e, plan->d_uv_kernel, plan->d_w_kernel,
                    (Cx<T>*)sdp_mem_data(vis));
            SDP_HIP_CHECK_LAUNCH(status);
        }
    }
    plan->num_w_planes[0] += 1 + last - first;
}

template<typename T, typename U>
void grid_impl(sdp_GridderWtowerUVW* plan, const sdp_Mem* vis,
        const sdp_Mem* uvws, const sdp_Mem* start_chs, const sdp_Mem* end_chs,
        double f0, double df, sdp_Mem* subgrid_image, int off_u, int off_v,
        int off_w, int64_t r0, int64_t r1, sdp_Error* status)
{
    ensure_scratch<T>(plan, status);
    if (*status) return;
    const int k = sizeof(T) == 8;
    const int S = plan->subgrid_size, ws = plan->w_support;
    const int64_t layer = (int64_t)S * S;
    T* stack = (T*)plan->d_scratch[k];
    T* fbuf = stack + 2 * layer * ws;
    double* wimg = (double*)(fbuf + 2 * layer);      // complex double
    const U* d_uvw = (const U*)sdp_mem_data_const(uvws);
    const int* d_s = (const int*)sdp_mem_data_const(start_chs);
    const int* d_e = (const int*)sdp_mem_data_const(end_chs);
    int first = 0, last = 0;
    if (!w_range<U>(plan, d_uvw, sdp_mem_shape_dim(uvws, 0), f0, df, d_s,
            d_e, off_w, &first, &last, status))
        return;
    SDP_HIP_CHECK(hipMemsetAsync(stack, 0, 2 * layer * ws * sizeof(T), 0),
            status);
    SDP_HIP_CHECK(hipMemsetAsync(wimg, 0, 2 * layer * sizeof(double), 0),
            status);
    const AnyView wv = {wimg, 3};
    const AnyView fv = {fbuf, sizeof(T) == 8 ? 3 : 2};
    WtParams p = base_params(plan, off_u, off_v, off_w, f0, df, r0, r1,
            sdp_mem_shape_dim(vis, 1));
    const unsigned blocks = (unsigned)((r1 - r0 + 255) / 256);
    int ring = 0;
    for (int w_plane = first; w_plane <= last && !*status; ++w_plane)
    {
        if (w_plane != first)
        {
            // w image = w image / w_pattern + IFFT(layer 0); clear layer 0,
            // which becomes the new last layer.
            wt_scale_inv(wv, wv, plan->d_w_pattern, 1, layer, status);
            T* l0 = stack + 2 * layer * ring;
            SDP_HIP_CHECK(hipMemcpyAsync(fbuf, l0, 2 * layer * sizeof(T),
                    hipMemcpyDeviceToDevice, 0), status);
            fft_shift<T>(plan, fbuf, false, status);
            wt_accum(wv, fv, nullptr, 0, layer, status);
            SDP_HIP_CHECK(hipMemsetAsync(l0, 0, 2 * layer * sizeof(T), 0),
                    status);
            ring = (ring + 1) % ws;
        }
        p.w_plane = w_plane;
        p.ring = ring;
        if (blocks)
        {
            k_wt_grid<T, U><<<blocks, 256>>>(p, (Cx<T>*)stack, d_uvw, d_s, d_e,
                    plan->d_uv_kernel, plan->d_w_kernel,
                    (const Cx<T>*)sdp_mem_data_const(vis));
            SDP_HIP_CHECK_LAUNCH(status);
        }
    }
    for (int i = 0; i < ws && !*status; ++i)
    {
        wt_scale_inv(wv, wv, plan->d_w_pattern, 1, layer, status);
        T* li = stack + 2 * layer * ((ring + i) % ws);
        SDP_HIP_CHECK(hipMemcpyAsync(fbuf, li, 2 * layer * sizeof(T),
                hipMemcpyDeviceToDevice, 0), status);
        fft_shift<T>(plan, fbuf, false, status);
        wt_accum(wv, fv, nullptr, 0, layer, status);
    }
    const AnyView out = {sdp_mem_data(subgrid_image),
            any_kind(sdp_mem_type(subgrid_image))};
    wt_accum(out, wv, plan->d_w_pattern, last + ws / 2 - 1, layer, status);
    plan->num_w_planes[1] += 1 + last - first;
}

// Shapes the kernels rely on (the reference indexes without checking; a
// mismatch here would address device memory outside the arrays).
bool shapes_ok(const sdp_GridderWtowerUVW* plan, const sdp_Mem* sub,
        const sdp_Mem* uvws, const sdp_Mem* s, const sdp_Mem* e,
        const sdp_Mem* vis, int64_t* start_row, int64_t* end_row)
{
    const int64_t rows = sdp_mem_shape_dim(uvws, 0);
    if (sdp_mem_num_dims(uvws) != 2 || sdp_mem_shape_dim(uvws, 1) != 3 ||
            sdp_mem_num_dims(vis) != 2 || sdp_mem_shape_dim(vis, 0) != rows ||
            sdp_mem_num_elements(s) != rows ||
            sdp_mem_num_elements(e) != rows ||
            sdp_mem_num_dims(sub) != 2 ||
            sdp_mem_shape_dim(sub, 0) != plan->subgrid_size ||
            sdp_mem_shape_dim(sub, 1) != plan->subgrid_size ||
            !sdp_mem_is_c_contiguous(uvws) || !sdp_mem_is_c_contiguous(vis) ||
            !sdp_mem_is_c_contiguous(sub) || !sdp_mem_is_c_contiguous(s) ||
            !sdp_mem_is_c_contiguous(e))
    {
        SDP_LOG_ERROR("Inconsistent array shapes: uvws must be [rows, 3], "
                "vis [rows, chans], start/end_chs [rows] and the sub-grid "
                "image [%d, %d], all C-contiguous", plan->subgrid_size,
                plan->subgrid_size);
        return false;
    }
    if (sdp_mem_type(s) != SDP_MEM_INT || sdp_mem_type(e) != SDP_MEM_INT)
    {
        SDP_LOG_ERROR("start_chs and end_chs must be int32");
        return false;
    }
    if (*start_row < 0 || *end_row < 0)
    {
        *start_row = 0;
        *end_row = rows;
    }
    *end_row = std::min(*end_row, rows);
    *start_row = std::min(*start_row, *end_row);
    return true;
}

// Type checks (.cpp:200-238): (c128, f64, c128), (c64, f64, c64),
// (c64, f32, c64) for (stack / vis, uvws, vis).
int type_combo(const sdp_Mem* uvws, const sdp_Mem* vis)
{
    const sdp_MemType tu = sdp_mem_type(uvws), tv = sdp_mem_type(vis);
    if (tv == SDP_MEM_COMPLEX_DOUBLE && tu == SDP_MEM_DOUBLE) return 0;
    if (tv == SDP_MEM_COMPLEX_FLOAT && tu == SDP_MEM_DOUBLE) return 1;
    if (tv == SDP_MEM_COMPLEX_FLOAT && tu == SDP_MEM_FLOAT) return 2;
    return -1;
}

bool same_location(std::initializer_list<const sdp_Mem*> mems)
{
    const sdp_MemLocation loc = sdp_mem_location(*mems.begin());
    for (const sdp_Mem* m : mems)
        if (sdp_mem_location(m) != loc) return false;
    return true;
}

void correct(sdp_GridderWtowerUVW* plan, sdp_Mem* facet, int off_l,
        int off_m, int w_offset, bool inverse, sdp_Error* status)
{
    if (*status) return;
    plan_ensure_correction(plan, status);
    const int kind = any_kind(sdp_mem_type(facet));
    if (kind < 0 || sdp_mem_num_dims(facet) != 2 ||
            !sdp_mem_is_c_contiguous(facet))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Facet must be a 2-D C-contiguous real or complex "
                "array");
        return;
    }
    Staged f;
    f.init(facet, status);
    if (*status) return;
    const int nl = (int)sdp_mem_shape_dim(facet, 0);
    const int nm = (int)sdp_mem_shape_dim(facet, 1);
    const AnyView v = {sdp_mem_data(f.dev), kind};
    const dim3 blocks((nm + 255) / 256, nl);
    k_grid_correct<<<blocks, 256>>>(v, nl, nm, off_l, off_m,
            corr_params(plan, w_offset, inverse));
    SDP_HIP_CHECK_LAUNCH(status);
    f.write_back(status);
}

} // namespace

namespace sdp_wt {

void plan_ensure_device(sdp_GridderWtowerUVW* plan, sdp_Error* status)
{
    if (*status) return;
    if (!sdp_hip::device_available())
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("No GPU available for the w-towers gridder.");
        return;
    }
    upload(*plan->uv_kernel, &plan->d_uv_kernel, status);
    upload(*plan->w_kernel, &plan->d_w_kernel, status);
    upload(*plan->w_pattern, &plan->d_w_pattern, status);
}

void plan_ensure_correction(sdp_GridderWtowerUVW* plan, sdp_Error* status)
{
    plan_ensure_device(plan, status);
    if (plan->d_pswf_lm || *status) return;
    upload(generate_pswf(plan->support * (M_PI / 2), plan->image_size, true),
            &plan->d_pswf_lm, status);
    const Pswf pn = make_pswf(plan->w_support * (M_PI / 2));
    upload(pn.coef, &plan->d_pswf_n, status);
    plan->n_pswf_n = (int)pn.coef.size();
}

CorrParams corr_params(const sdp_GridderWtowerUVW* plan, int w_offset,
        bool inverse)
{
    CorrParams cp;
    cp.image_size = plan->image_size;
    cp.theta = plan->theta;
    cp.w_step = plan->w_step;
    cp.shear_u = plan->shear_u;
    cp.shear_v = plan->shear_v;
    cp.pswf_lm = plan->d_pswf_lm;
    cp.pswf_n = plan->d_pswf_n;
    cp.n_pswf_n = plan->n_pswf_n;
    cp.c_n = plan->w_support * (M_PI / 2);
    cp.w_offset = w_offset;
    cp.inverse = inverse ? 1 : 0;
    cp.pn_tab = nullptr;
    cp.scale_f64 = nullptr;
    cp.scale_f32 = nullptr;
    return cp;
}

} // namespace sdp_wt

extern "C" {

sdp_GridderWtowerUVW* sdp_gridder_wtower_uvw_create(int image_size,
        int subgrid_size, double theta, double w_step, double shear_u,
        double shear_v, int support, int oversampling, int w_support,
        int w_oversampling, sdp_Error* status)
{
    if (*status) return nullptr;
    if (subgrid_size % 2 != 0)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Subgrid size must be even (value given was %d).",
                subgrid_size);
        return nullptr;
    }
    sdp_GridderWtowerUVW* plan = (sdp_GridderWtowerUVW*)calloc(1,
            sizeof(sdp_GridderWtowerUVW));
    plan->image_size = image_size;
    plan->subgrid_size = subgrid_size;
    plan->theta = theta;
    plan->w_step = w_step;
    plan->shear_u = shear_u;
    plan->shear_v = shear_v;
    plan->support = support;
    plan->oversampling = oversampling;
    plan->w_support = w_support;
    plan->w_oversampling = w_oversampling;
    plan->uv_kernel = new std::vector<double>(
            make_pswf_kernel(support, oversampling));
    plan->w_kernel = new std::vector<double>(
            make_pswf_kernel(w_support, w_oversampling));
    const std::vector<std::complex<double> > wp = make_w_pattern(subgrid_size,
            theta, shear_u, shear_v, w_step);
    plan->w_pattern = new std::vector<double>(2 * wp.size());
    memcpy(plan->w_pattern->data(), wp.data(), wp.size() * 16);
    return plan;
}

void sdp_gridder_wtower_uvw_free(sdp_GridderWtowerUVW* plan)
{
    if (!plan) return;
    delete plan->uv_kernel;
    delete plan->w_kernel;
    delete plan->w_pattern;
    // Device buffers exist only if the plan was used (no HIP call for a
    // plan that never ran, e.g. in a CPU-only process).
    void* dev[] = {plan->d_uv_kernel, plan->d_w_kernel, plan->d_w_pattern,
            plan->d_pswf_lm, plan->d_pswf_n, plan->d_scratch[0],
            plan->d_scratch[1]};
    for (void* p : dev)
        if (p) (void)hipFree(p);
    for (int k = 0; k < 2; ++k)
        if (plan->fft[k]) sdp_fft::destroy_2d(plan->fft[k]);
    free(plan);
}

void sdp_gridder_wtower_uvw_degrid(sdp_GridderWtowerUVW* plan,
        const sdp_Mem* subgrid_image, int subgrid_offset_u,
        int subgrid_offset_v, int subgrid_offset_w, double freq0_hz,
        double dfreq_hz, const sdp_Mem* uvws, const sdp_Mem* start_chs,
        const sdp_Mem* end_chs, sdp_Mem* vis, int64_t start_row,
        int64_t end_row, sdp_Error* status)
{
    if (*status) return;
    if (dfreq_hz == 0.0) dfreq_hz = 10;   // .cpp:743
    if (!same_location({vis, subgrid_image, uvws, start_chs, end_chs}))
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("All arrays must be in the same memory space");
        return;
    }
    if (!shapes_ok(plan, subgrid_image, uvws, start_chs, end_chs, vis,
            &start_row, &end_row))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    const int combo = type_combo(uvws, vis);
    const int ks = any_kind(sdp_mem_type(subgrid_image));
    if (combo < 0 || ks < 0)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data types: subgrids has type %s; uvws "
                "has type %s; vis has type %s",
                sdp_mem_type_name(sdp_mem_type(subgrid_image)),
                sdp_mem_type_name(sdp_mem_type(uvws)),
                sdp_mem_type_name(sdp_mem_type(vis)));
        return;
    }
    // The image is scaled into the vis precision (scale_inv_array
    // combinations, utils.cpp:1557-1592).
    if ((combo == 0) != (ks == 1 || ks == 3))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported image data type");
        return;
    }
    plan_ensure_device(plan, status);
    Staged sg, uv, s, e, v;
    sg.init(subgrid_image, status);
    uv.init(uvws, status);
    s.init(start_chs, status);
    e.init(end_chs, status);
    v.init(vis, status);
    if (*status) return;
    if (combo == 0)
        degrid_impl<double, double>(plan, sg.dev, subgrid_offset_u,
                subgrid_offset_v, subgrid_offset_w, freq0_hz, dfreq_hz,
                uv.dev, s.dev, e.dev, v.dev, start_row, end_row, status);
    else if (combo == 1)
        degrid_impl<float, double>(plan, sg.dev, subgrid_offset_u,
                subgrid_offset_v, subgrid_offset_w, freq0_hz, dfreq_hz,
                uv.dev, s.dev, e.dev, v.dev, start_row, end_row, status);
    else
        degrid_impl<float, float>(plan, sg.dev, subgrid_offset_u,
                subgrid_offset_v, subgrid_offset_w, freq0_hz, dfreq_hz,
                uv.dev, s.dev, e.dev, v.dev, start_row, end_row, status);
    v.write_back(status);
}

void sdp_gridder_wtower_uvw_grid(sdp_GridderWtowerUVW* plan,
        const sdp_Mem* vis, const sdp_Mem* uvws, const sdp_Mem* start_chs,
        const sdp_Mem* end_chs, double freq0_hz, double dfreq_hz,
        sdp_Mem* subgrid_image, int subgrid_offset_u, int subgrid_offset_v,
        int subgrid_offset_w, int64_t start_row, int64_t end_row,
        sdp_Error* status)
{
    if (*status) return;
    if (dfreq_hz == 0.0) dfreq_hz = 10;   // .cpp:953
    if (!same_location({vis, subgrid_image, uvws, start_chs, end_chs}))
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("All arrays must be in the same memory space");
        return;
    }
    if (!shapes_ok(plan, subgrid_image, uvws, start_chs, end_chs, vis,
            &start_row, &end_row))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    const int combo = type_combo(uvws, vis);
    if (combo < 0 || any_kind(sdp_mem_type(subgrid_image)) < 0)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data types: subgrids has type %s; uvws "
                "has type %s; vis has type %s",
                sdp_mem_type_name(sdp_mem_type(subgrid_image)),
                sdp_mem_type_name(sdp_mem_type(uvws)),
                sdp_mem_type_name(sdp_mem_type(vis)));
        return;
    }
    plan_ensure_device(plan, status);
    Staged sg, uv, s, e, v;
    sg.init(subgrid_image, status);
    uv.init(uvws, status);
    s.init(start_chs, status);
    e.init(end_chs, status);
    v.init(vis, status);
    if (*status) return;
    if (combo == 0)
        grid_impl<double, double>(plan, v.dev, uv.dev, s.dev, e.dev, freq0_hz,
                dfreq_hz, sg.dev, subgrid_offset_u, subgrid_offset_v,
                subgrid_offset_w, start_row, end_row, status);
    else if (combo == 1)
        grid_impl<float, double>(plan, v.dev, uv.dev, s.dev, e.dev, freq0_hz,
                dfreq_hz, sg.dev, subgrid_offset_u, subgrid_offset_v,
                subgrid_offset_w, start_row, end_row, status);
    else
        grid_impl<float, float>(plan, v.dev, uv.dev, s.dev, e.dev, freq0_hz,
                dfreq_hz, sg.dev, subgrid_offset_u, subgrid_offset_v,
                subgrid_offset_w, start_row, end_row, status);
    sg.write_back(status);
}

void sdp_gridder_wtower_uvw_grid_correct(sdp_GridderWtowerUVW* plan,
        sdp_Mem* facet, int facet_offset_l, int facet_offset_m, int w_offset,
        sdp_Error* status)
{
    correct(plan, facet, facet_offset_l, facet_offset_m, w_offset, true,
            status);
}

void sdp_gridder_wtower_uvw_degrid_correct(sdp_GridderWtowerUVW* plan,
        sdp_Mem* facet, int facet_offset_l, int facet_offset_m, int w_offset,
        sdp_Error* status)
{
    correct(plan, facet, facet_offset_l, facet_offset_m, w_offset, false,
            status);
}

int sdp_gridder_wtower_uvw_num_w_planes(const sdp_GridderWtowerUVW* plan,
        int gridding)
{
    return plan->num_w_planes[gridding ? 1 : 0];
}

int sdp_gridder_wtower_uvw_image_size(const sdp_GridderWtowerUVW* plan)
{
    return plan->image_size;
}

int sdp_gridder_wtower_uvw_oversampling(const sdp_GridderWtowerUVW* plan)
{
    return plan->oversampling;
}

double sdp_gridder_wtower_uvw_shear_u(const sdp_GridderWtowerUVW* plan)
{
    return plan->shear_u;
}

double sdp_gridder_wtower_uvw_shear_v(const sdp_GridderWtowerUVW* plan)
{
    return plan->shear_v;
}

int sdp_gridder_wtower_uvw_subgrid_size(const sdp_GridderWtowerUVW* plan)
{
    return plan->subgrid_size;
}

int sdp_gridder_wtower_uvw_support(const sdp_GridderWtowerUVW* plan)
{
    return plan->support;
}

double sdp_gridder_wtower_uvw_theta(const sdp_GridderWtowerUVW* plan)
{
    return plan->theta;
}

int sdp_gridder_wtower_uvw_w_oversampling(const sdp_GridderWtowerUVW* plan)
{
    return plan->w_oversampling;
}

double sdp_gridder_wtower_uvw_w_step(const sdp_GridderWtowerUVW* plan)
{
    return plan->w_step;
}

int sdp_gridder_wtower_uvw_w_support(const sdp_GridderWtowerUVW* plan)
{
    return plan->w_support;
}

} // extern "C"
