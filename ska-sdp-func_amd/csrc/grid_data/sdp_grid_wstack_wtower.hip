// MI355X-native w-stacking x w-towers imaging driver
// (sdp_grid_wstack_wtower.cpp of ska-sdp-func 1.2.2: degrid_all :218-472,
// grid_all :475-736).
//
// Reference structure: for every w-stack plane iw, channel clamps over all
// rows select the plane's visibilities; for every sub-grid (iu, iv) a
// second clamp over all rows selects the sub-grid's visibilities
// (count_visibilities, O(rows x sub-grids)); sub-grid tasks then run one
// after the other through sdp_gridder_wtower_uvw_(de)grid, each moving a
// w_support-deep stack through its own w-layers with one S x S FFT per
// layer.
//
// Here:
//  1. Binning (k_bin): one pass over the rows evaluates, with the
//     reference's own clamp arithmetic, which (w-stack plane, sub-grid,
//     w-layer) every channel run of every row belongs to, including the
//     sub-grid bounds check of the (de)gridding kernel. Items are sorted by
//     (plane group, w-layer, sub-grid slot) with a device radix sort.
//  2. Towers: all sub-grids of a w-stack plane (up to a memory budget per
//     group) move through the w-layers in lock step. A visibility's
//     contribution does not depend on where its tower starts or ends (the
//     w-pattern exponents cancel), so one common layer range
//     per group replaces the per-task ranges. Per layer: one batched S x S
//     rocFFT over the group and one fused element-wise pass; the FFT-shift
//     checkerboards are folded into the neighbouring passes (exact sign
//     flips).
//  3. (De)gridding kernels: one wavefront per item, lanes over the uv taps,
//     looping over the w_support layers (512 taps per visibility at
//     support 8); gridding adds with device atomics into the stack.
//  4. Image side per w-stack plane: one gather pass sums the sub-grids into
//     the full grid in the reference's task order (no atomics, no zeroing),
//     one G x G rocFFT, one fused pass for normalisation, grid correction
//     and image accumulation (and the mirror for degridding).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "utility/wave_ops.h"
#include "ska-sdp-func/grid_data/sdp_grid_wstack_wtower.h"
#include "ska-sdp-func/grid_data/sdp_gridder_wtower_uvw.h"
#include "wtower_dev.h"
#include "wtower_ops.h"
#include "wtower_plan.h"
#include "../fft/fft2d.h"
#include "es_fft.h"
#include "es_fft_wstack.h"
#include "../utility/sdp_hip.h"

using namespace sdp_wt;

namespace {

constexpr int kWaves = 4;            // wavefronts per (de)gridding block

// ---------------------------------------------------------------------------
// Geometry of one call (sdp_grid_wstack_wtower.cpp:297-330 / 567-602).
struct Geo
{
    double f0, df;
    int64_t num_rows, num_chan;
    int S, eff, support, w_support;
    double theta, w_step, H, eff_dist, ws_dist;
    int64_t min_iu, max_iu, min_iv, max_iv, min_iw, max_iw;
    int64_t nu, nv, niw, ntask;
    int64_t P0, NP;                  // global w-layer index base and count
    int plane_offset, plane_stride;
    // Plane set (extension): when plane_mask is set, plane iw is processed
    // iff plane_mask[clamp(iw - mask_first, 0, mask_n - 1)] != 0 (offset /
    // stride are then ignored): a plane below or above the mask's range
    // belongs to the owner of the first or last entry, so masks that
    // partition the range partition every plane and no visibility is lost
    // if the caller's range model misses one. Device memory.
    const int* plane_mask;
    int64_t mask_first, mask_n;
    int fused;                       // sort runs by (group, slot, layer)
};

// Whether the call processes w-stack plane iw (absolute index).
__host__ __device__ __forceinline__ bool plane_selected(const Geo& g,
        int64_t iw)
{
    if (g.plane_mask)
    {
        int64_t m = iw - g.mask_first;
        m = m < 0 ? 0 : (m >= g.mask_n ? g.mask_n - 1 : m);
        return g.mask_n > 0 && g.plane_mask[m] != 0;
    }
    return (iw - g.min_iw) % g.plane_stride == g.plane_offset;
}

// sdp_gridder_clamp_channels_single / _uv row arithmetic
// (sdp_gridder_clamp_channels.cpp:37-62).
__device__ __forceinline__ void clamp_rows(double x, double f0, double df,
        int s_in, int e_in, double lo, double hi, int* s_out, int* e_out)
{
#pragma clang fp contract(off)
    const double x0 = x * (f0 / kC0);
    const double dx = x * (df / kC0);
    const double eta = fmax(fabs(lo - x0), fabs(hi - x0)) / 2147483645.0;
    int s, e;
    if (fabs(dx) > eta)
    {
        const int mins = (int)(int64_t)ceil((lo - x0) / dx);
        const int maxs = (int)(int64_t)ceil((hi - x0) / dx);
        const bool pos = dx > 0;
        s = max(s_in, pos ? mins : maxs);
        e = min(e_in, pos ? maxs : mins);
    }
    else if (lo > x0 || hi <= x0)
    {
        s = 0;
        e = 0;
    }
    else
    {
        s = s_in;
        e = e_in;
    }
    *s_out = s;
    *e_out = max(e, s);
}

// Candidate index range of x_c = x (f0 + c df) / c0 over channels [s, e)
// for cells [i d - d/2, (i+1) d - d/2), one cell of margin on each side.
__device__ __forceinline__ void cell_range(double x, double f0, double df,
        int s, int e, double d, int64_t lo_lim, int64_t hi_lim, int64_t* lo,
        int64_t* hi)
{
    const double a = f0 * x / kC0 + s * (df * x / kC0);
    const double b = f0 * x / kC0 + (e - 1) * (df * x / kC0);
    const double mn = fmin(a, b), mx = fmax(a, b);
    *lo = max((int64_t)floor(mn / d + 0.5) - 1, lo_lim);
    *hi = min((int64_t)floor(mx / d + 0.5) + 1, hi_lim);
}

// Task slot of (w-stack plane, sub-grid) after host assignment.
struct Slot
{
    int group, slot;
};

struct BinOut
{
    // count pass
    int64_t* row_count;
    unsigned char* occupied;         // [niw][ntask]
    // emit pass
    const int64_t* row_offset;
    const Slot* slot_map;            // [niw][ntask]
    uint64_t* keys;
    uint32_t* idx;
    int4* items;                     // row, c0, c1, slot (unsorted)
    unsigned int* hist;              // [groups][NP]
    int64_t t_cap;
};

// One pass over the rows: every channel run of every row that the
// reference would (de)grid, with its w-stack plane, sub-grid and w-layer.
template<typename U, bool EMIT>
__global__ void k_bin(const U* __restrict__ uvw, Geo g, BinOut out)
{
#pragma clang fp contract(off)
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= g.num_rows) return;
    const double u = (double)uvw[3 * r];
    const double v = (double)uvw[3 * r + 1];
    const double w = (double)uvw[3 * r + 2];
    const int C = (int)g.num_chan;
    int64_t pos = EMIT ? out.row_offset[r] : 0;
    int64_t count = 0;
    int64_t iw_lo, iw_hi;
    cell_range(w, g.f0, g.df, 0, C, g.ws_dist, g.min_iw, g.max_iw, &iw_lo,
            &iw_hi);
    for (int64_t iw = iw_lo; iw <= iw_hi; ++iw)
    {
        if (!plane_selected(g, iw)) continue;
        const int64_t iw_rel = iw - g.min_iw;
        // Visibilities on the w-stack plane (.cpp:336-343 / 612-618).
        const double min_w = iw * g.ws_dist - g.ws_dist / 2;
        const double max_w = (iw + 1) * g.ws_dist - g.ws_dist / 2;
        int sw, ew;
        clamp_rows(w, g.f0, g.df, 0, C, min_w, max_w, &sw, &ew);
        if (sw >= ew) continue;
        const int off_w = (int)(iw * g.H);
        int64_t iu_lo, iu_hi;
        cell_range(u, g.f0, g.df, sw, ew, g.eff_dist, g.min_iu, g.max_iu,
                &iu_lo, &iu_hi);
        for (int64_t iu = iu_lo; iu <= iu_hi; ++iu)
        {
            // Sub-grid selection (clamp_channels_uv, .cpp:399-406).
            const double min_u = iu * g.eff_dist - g.eff_dist / 2;
            const double max_u = (iu + 1) * g.eff_dist - g.eff_dist / 2;
            int su, eu;
            clamp_rows(u, g.f0, g.df, sw, ew, min_u, max_u, &su, &eu);
            if (su >= eu) continue;
            int64_t iv_lo, iv_hi;
            cell_range(v, g.f0, g.df, su, eu, g.eff_dist, g.min_iv, g.max_iv,
                    &iv_lo, &iv_hi);
            for (int64_t iv = iv_lo; iv <= iv_hi; ++iv)
            {
                const double min_v = iv * g.eff_dist - g.eff_dist / 2;
                const double max_v = (iv + 1) * g.eff_dist - g.eff_dist / 2;
                int sv, ev;
                clamp_rows(v, g.f0, g.df, su, eu, min_v, max_v, &sv, &ev);
                if (sv >= ev) continue;
                const int64_t task = (iu - g.min_iu) * g.nv + (iv - g.min_iv);
                if (!EMIT)
                    out.occupied[iw_rel * g.ntask + task] = 1;
                Slot sl = {0, 0};
                if (EMIT) sl = out.slot_map[iw_rel * g.ntask + task];
                const int off_u = (int)(iu * g.eff);
                const int off_v = (int)(iv * g.eff);
                // w-layers of the tower (sdp_gridder_wtower_uvw.cpp:95-119).
                const double s_uvw0 = g.f0 / kC0, s_duvw = g.df / kC0;
                double uvw0[3] = {u * s_uvw0, v * s_uvw0, w * s_uvw0};
                const double duvw[3] = {u * s_duvw, v * s_duvw, w * s_duvw};
                uvw0[0] -= off_u / g.theta;
                uvw0[1] -= off_v / g.theta;
                const double wa = w * s_uvw0 + sv * duvw[2];
                const double wb = w * s_uvw0 + (ev - 1) * duvw[2];
                const int64_t p_lo = (int64_t)floor(fmin(wa, wb) / g.w_step);
                const int64_t p_hi = (int64_t)floor(fmax(wa, wb) / g.w_step)
                        + 2;
                for (int64_t P = p_lo; P <= p_hi; ++P)
                {
                    const int64_t w_plane = P - off_w;
                    int64_t sp = sv, ep = ev;
                    const double pmin = (w_plane + off_w - 1) * g.w_step;
                    const double pmax = (w_plane + off_w) * g.w_step;
                    clamp_inline(w, g.f0, g.df, &sp, &ep, pmin, pmax);
                    if (sp >= ep) continue;
                    // Sub-grid bounds check of the (de)gridding kernel.
                    const int half = g.S / 2;
                    const double u_min = floor(g.theta * (uvw0[0] +
                            sp * duvw[0]));
                    const double u_max = ceil(g.theta * (uvw0[0] +
                            (ep - 1) * duvw[0]));
                    const double v_min = floor(g.theta * (uvw0[1] +
                            sp * duvw[1]));
                    const double v_max = ceil(g.theta * (uvw0[1] +
                            (ep - 1) * duvw[1]));
                    if (u_min < -half || u_max >= half || v_min < -half ||
                            v_max >= half)
                        continue;
                    const int64_t p_rel = P - g.P0;
                    if (p_rel < 0 || p_rel >= g.NP) continue;  // (never)
                    if (EMIT)
                    {
                        const uint64_t key = g.fused ?
                                ((uint64_t)sl.group * out.t_cap + sl.slot) *
                                g.NP + p_rel :
                                ((uint64_t)sl.group * g.NP + p_rel) *
                                out.t_cap + sl.slot;
                        out.keys[pos] = key;
                        out.idx[pos] = (uint32_t)pos;
                        out.items[pos] = make_int4((int)r, (int)sp, (int)ep,
                                sl.slot);
                        atomicAdd(&out.hist[sl.group * g.NP + p_rel], 1u);
                        ++pos;
                    }
                    ++count;
                }
            }
        }
    }
    if (!EMIT) out.row_count[r] = count;
}

// First n entries = a, next n = b.
__global__ void k_fill_int(int* p, int64_t n, int a, int b)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < 2 * n) p[i] = (i < n) ? a : b;
}

__global__ void k_gather_items(const uint32_t* __restrict__ idx,
        const int4* __restrict__ in, int4* __restrict__ out, int64_t n)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[idx[i]];
}

// ---------------------------------------------------------------------------
// Per-group parameters of the tower kernels.
struct TowerParams
{
    int S, support, w_support, os, wos;
    double theta, w_step, f0, df;
    int64_t num_chan;
    int off_w, w_plane, ring;
    int64_t layer;                   // S * S
    int64_t layer_stride;            // slots_alloc * S * S (layer-major)
    const int* task;                 // slot -> task id
    int64_t nv, min_iu, min_iv;
    int eff;
};

__device__ __forceinline__ int parity_sign(int64_t a)
{
    return (a & 1) ? -1 : 1;
}

struct Taps2
{
    int iu0, iv0, u_off, v_off, w_off;
    bool valid;
};

// Kernel offsets of channel c (sdp_gridder_wtower_uvw.cpp:121-141).
template<typename U>
__device__ __forceinline__ Taps2 item_taps(const TowerParams& p,
        const U* __restrict__ uvws, int row, int c, int off_u, int off_v)
{
#pragma clang fp contract(off)
    const double s_uvw0 = p.f0 / kC0, s_duvw = p.df / kC0;
    const double uvw[3] = {(double)uvws[3 * (int64_t)row],
            (double)uvws[3 * (int64_t)row + 1],
            (double)uvws[3 * (int64_t)row + 2]};
    double uvw0[3] = {uvw[0] * s_uvw0, uvw[1] * s_uvw0, uvw[2] * s_uvw0};
    const double duvw[3] = {uvw[0] * s_duvw, uvw[1] * s_duvw,
            uvw[2] * s_duvw};
    uvw0[0] -= off_u / p.theta;
    uvw0[1] -= off_v / p.theta;
    uvw0[2] -= ((p.off_w + p.w_plane - 1) * p.w_step);
    const double uu = uvw0[0] + c * duvw[0];
    const double vv = uvw0[1] + c * duvw[1];
    const double ww = uvw0[2] + c * duvw[2];
    const double theta_ov = p.theta * p.os;
    const double w_step_ov = 1.0 / p.w_step * p.wos;
    const int half_ov = (p.S / 2 - p.support / 2 + 1) * p.os;
    const int iu0_ov = int(round(uu * theta_ov)) + half_ov;
    const int iv0_ov = int(round(vv * theta_ov)) + half_ov;
    const int iw0_ov = int(round(ww * w_step_ov));
    Taps2 t;
    t.iu0 = iu0_ov / p.os;
    t.iv0 = iv0_ov / p.os;
    t.u_off = (iu0_ov % p.os) * p.support;
    t.v_off = (iv0_ov % p.os) * p.support;
    t.w_off = (iw0_ov % p.wos) * p.w_support;
    t.valid = iu0_ov >= 0 && iv0_ov >= 0 && iw0_ov >= 0;
    return t;
}

// Offset of stack cell (layer iw of the tower, row iu, column iv) from the
// slot's base, following the reference's flat [w_support, S, S] indexing
// through the ring (see stack_cell in sdp_gridder_wtower_uvw.hip); -1
// outside. The stack is layer-major: [w_support][slots][S][S], so that one
// layer of all sub-grids is a contiguous FFT batch. *sign = checkerboard
// sign of the cell.
__device__ __forceinline__ int64_t tower_cell(const TowerParams& p, int iw,
        int iu, int iv, int* sign)
{
    if (iu >= 0 && iu < p.S && iv >= 0 && iv < p.S)
    {
        *sign = parity_sign(iu + iv);
        return ((p.ring + iw) % p.w_support) * p.layer_stride +
                (int64_t)iu * p.S + iv;
    }
    const int64_t f = ((int64_t)iw * p.S + iu) * p.S + iv;
    if (f < 0 || f >= p.w_support * p.layer) return -1;
    const int l = (int)(f / p.layer);
    const int64_t rem = f - l * p.layer;
    *sign = parity_sign(rem / p.S + rem % p.S);
    return ((p.ring + l) % p.w_support) * p.layer_stride + rem;
}

template<typename T>
__device__ __forceinline__ T wave_sum(T x)
{
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// Degrid: one wavefront per item; vis[row, c] += sum over the taps of the
// checkerboard-corrected stack (sdp_gridder_wtower_uvw.cpp:143-171).
template<typename T, typename U>
__global__ __launch_bounds__(64 * kWaves)
void k_tower_degrid(TowerParams p, const int4* __restrict__ items,
        int64_t n_items, const U* __restrict__ uvws,
        const Cx<T>* __restrict__ stack, const double* __restrict__ uv_kernel,
        const double* __restrict__ w_kernel, Cx<T>* __restrict__ vis)
{
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const int64_t it = blockIdx.x * (int64_t)kWaves + (threadIdx.x >> 6);
    if (it >= n_items) return;
    const int4 item = items[it];
    const int task = p.task[item.w];
    const int off_u = (int)((p.min_iu + task / p.nv) * p.eff);
    const int off_v = (int)((p.min_iv + task % p.nv) * p.eff);
    const Cx<T>* base = stack + item.w * p.layer;
    const int taps = p.support * p.support;
    for (int c = item.y; c < item.z; ++c)
    {
        const Taps2 t = item_taps(p, uvws, item.x, c, off_u, off_v);
        if (!t.valid) continue;
        Cx<T> acc = cx<T>(0, 0);
        for (int k = lane; k < taps; k += 64)
        {
            const int iu = k / p.support, iv = k % p.support;
            const T ku = (T)uv_kernel[t.u_off + iu];
            const T kv = (T)uv_kernel[t.v_off + iv];
            for (int iw = 0; iw < p.w_support; ++iw)
            {
                int sgn = 1;
                const int64_t cell = tower_cell(p, iw, t.iu0 + iu,
                        t.iv0 + iv, &sgn);
                if (cell < 0) continue;
                const Cx<T> gv = base[cell];
                const T kw = (T)w_kernel[t.w_off + iw];
                const T gr = sgn < 0 ? -gv.re : gv.re;
                const T gi = sgn < 0 ? -gv.im : gv.im;
                acc.re += kw * (ku * (kv * gr));
                acc.im += kw * (ku * (kv * gi));
            }
        }
        acc.re = wave_sum(acc.re);
        acc.im = wave_sum(acc.im);
        if (lane == 0)
        {
            Cx<T>& out = vis[(int64_t)item.x * p.num_chan + c];
            out.re += acc.re;
            out.im += acc.im;
        }
    }
}

// Grid: one wavefront per item; the taps are added with device atomics to
// the stack, pre-multiplied by the checkerboard of the inverse FFT that
// follows (sdp_gridder_wtower_uvw.cpp:455-480).
template<typename T, typename U>
__global__ __launch_bounds__(64 * kWaves)
void k_tower_grid(TowerParams p, const int4* __restrict__ items,
        int64_t n_items, const U* __restrict__ uvws, Cx<T>* __restrict__ stack,
        const double* __restrict__ uv_kernel,
        const double* __restrict__ w_kernel, const Cx<T>* __restrict__ vis)
{
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const int64_t it = blockIdx.x * (int64_t)kWaves + (threadIdx.x >> 6);
    if (it >= n_items) return;
    const int4 item = items[it];
    const int task = p.task[item.w];
    const int off_u = (int)((p.min_iu + task / p.nv) * p.eff);
    const int off_v = (int)((p.min_iv + task % p.nv) * p.eff);
    Cx<T>* base = stack + item.w * p.layer;
    const int taps = p.support * p.support;
    for (int c = item.y; c < item.z; ++c)
    {
        const Taps2 t = item_taps(p, uvws, item.x, c, off_u, off_v);
        if (!t.valid) continue;
        const Cx<T> v = vis[(int64_t)item.x * p.num_chan + c];
        for (int k = lane; k < taps; k += 64)
        {
            const int iu = k / p.support, iv = k % p.support;
            const T ku = (T)uv_kernel[t.u_off + iu];
            const T kv = (T)uv_kernel[t.v_off + iv];
            for (int iw = 0; iw < p.w_support; ++iw)
            {
                int sgn = 1;
                const int64_t cell = tower_cell(p, iw, t.iu0 + iu,
                        t.iv0 + iv, &sgn);
                if (cell < 0) continue;
                const T kw = (T)w_kernel[t.w_off + iw];
                const T wr = kw * v.re, wi = kw * v.im;
                const T ur = ku * wr, ui = ku * wi;
                T ar = kv * ur, ai = kv * ui;
                if (sgn < 0)
                {
                    ar = -ar;
                    ai = -ai;
                }
                unsafeAtomicAdd(&base[cell].re, ar);
                unsafeAtomicAdd(&base[cell].im, ai);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Element-wise tower passes over `slots` sub-grids of S x S.

__device__ __forceinline__ Cx<double> pattern_pow(const Cx<double>* wp,
        int64_t i, int e)
{
    return (e == 1) ? wp[i] : cpow_int(wp[i], e);
}

// Gridding, one layer: wimg = wimg / D + checkerboard(IFFT(layer));
// layer = 0 (.cpp:1029-1058).
template<typename T>
__global__ void k_grid_step(Cx<double>* __restrict__ wimg,
        Cx<T>* __restrict__ layer_base, const Cx<double>* __restrict__ wp,
        int64_t layer, int S, int64_t n, int clear)
{
#pragma clang fp contract(off)
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t e = i % layer;
    Cx<T>* l = layer_base + i;
    Cx<double> z = cdiv(wimg[i], wp[e]);
    const int sgn = parity_sign(e / S + e % S);
    const Cx<T> f = *l;
    z.re += (double)(sgn < 0 ? -f.re : f.re);
    z.im += (double)(sgn < 0 ? -f.im : f.im);
    wimg[i] = z;
    if (clear) *l = cx<T>(0, 0);
}

// Gridding, end of tower: sub-grid = (T)(wimg * D^e) with the checkerboard
// of the forward FFT that follows, written to layer 0 of the slot
// (.cpp:1102-1113 and sdp_fft_exec_shift).
template<typename T>
__global__ void k_grid_final(const Cx<double>* __restrict__ wimg,
        Cx<T>* __restrict__ out, const Cx<double>* __restrict__ wp,
        int64_t layer, int S, int e_final, int64_t n)
{
#pragma clang fp contract(off)
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t e = i % layer;
    Cx<double> z = wimg[i];
    if (e_final != 0) z = cmul(z, pattern_pow(wp, e, e_final));
    T re = (T)z.re, im = (T)z.im;
    if (parity_sign(e / S + e % S) < 0)
    {
        re = -re;
        im = -im;
    }
    out[i] = cx<T>(re, im);
}

// Degridding, start of tower: wimg = (c128)(checkerboard(IFFT(cut-out)) *
// norm) / D^e0 (.cpp:423-427 and :803-808).
template<typename T>
__global__ void k_degrid_init(Cx<T>* __restrict__ wimg,
        const Cx<double>* __restrict__ wp, int64_t layer, int S, T norm,
        int e0, int64_t n)
{
#pragma clang fp contract(off)
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t e = i % layer;
    Cx<T> x = wimg[i];
    if (parity_sign(e / S + e % S) < 0)
    {
        x.re = -x.re;
        x.im = -x.im;
    }
    x.re *= norm;
    x.im *= norm;
    const Cx<double> z = cdiv(cx<double>((double)x.re, (double)x.im),
            pattern_pow(wp, e, e0));
    wimg[i] = cx<T>((T)z.re, (T)z.im);
}

// Degridding, one layer: layer = checkerboard(wimg) (the forward FFT
// follows); wimg = wimg / D (.cpp:831-857).
template<typename T>
__global__ void k_degrid_step(Cx<T>* __restrict__ wimg,
        Cx<T>* __restrict__ layer_base, const Cx<double>* __restrict__ wp,
        int64_t layer, int S, int64_t n)
{
#pragma clang fp contract(off)
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t e = i % layer;
    const Cx<T> x = wimg[i];
    const bool neg = parity_sign(e / S + e % S) < 0;
    layer_base[i] = cx<T>(neg ? -x.re : x.re, neg ? -x.im : x.im);
    const Cx<double> z = cdiv(cx<double>((double)x.re, (double)x.im), wp[e]);
    wimg[i] = cx<T>((T)z.re, (T)z.im);
}

// Degridding: cut the sub-grids out of the FFT'd grid
// (sdp_gridder_subgrid_cut_out, utils.cpp:603-649) with the grid FFT's
// output checkerboard and the sub-grid IFFT's input checkerboard; slots
// [slots, slots_alloc) are zeroed. Grid: x = slot * nbx + column block,
// y = block of kCutRows sub-grid rows (one per thread iteration, their loads
// issued together: the kernel is bound by memory latency), so no
// per-element division; the slot's grid offsets (mod G) are uniform per
// block.
constexpr int kCutRows = 4;

template<typename T>
__global__ void k_cut_out(const Cx<T>* __restrict__ grid, int64_t G,
        Cx<T>* __restrict__ wimg, int S, int64_t layer, const int* task,
        int64_t nv, int64_t min_iu, int64_t min_iv, int eff, int64_t slots,
        int nbx, int perm_n2)
{
    const int64_t slot = blockIdx.x / nbx;
    const int b = (int)(blockIdx.x % nbx) * (int)blockDim.x + (int)threadIdx.x;
    const int a0 = (int)blockIdx.y * kCutRows;
    if (b >= S) return;
    Cx<T>* out = wimg + slot * layer + b;
    if (slot >= slots)
    {
#pragma unroll
        for (int r = 0; r < kCutRows; ++r)
            if (a0 + r < S) out[(int64_t)(a0 + r) * S] = cx<T>(0, 0);
        return;
    }
    // 32-bit index arithmetic (G < 2^30, tasks < 2^31; host-checked): the
    // int64 divisions here were ~450 scalar instructions per wave.
    const int t = task[slot];
    const int Gi = (int)G, nvi = (int)nv;
    const int q = t / nvi;
    const int iu = (int)min_iu + q, iv = (int)min_iv + (t - q * nvi);
    int ou = (Gi / 2 - S / 2 + iu * eff) % Gi;
    int ov = (Gi / 2 - S / 2 + iv * eff) % Gi;
    if (ou < 0) ou += Gi;
    if (ov < 0) ov += Gi;
    int64_t gv = ov + b;                  // b < S <= G
    if (gv >= G) gv -= G;
    Cx<T> x[kCutRows];
#pragma unroll
    for (int r = 0; r < kCutRows; ++r)
    {
        int64_t gu = ou + a0 + r;
        if (gu >= G) gu -= G;
        // Row gu of the FFT'd grid (stored permuted by the fused FFT).
        x[r] = (a0 + r < S) ?
                grid[sdp_es::fft_perm_row(gu, G, perm_n2) * G + gv] :
                cx<T>(0, 0);
    }
#pragma unroll
    for (int r = 0; r < kCutRows; ++r)
    {
        const int a = a0 + r;
        if (a >= S) break;
        int64_t gu = ou + a;
        if (gu >= G) gu -= G;
        const bool neg = ((gu + gv + a + b) & 1) != 0;
        out[(int64_t)a * S] = cx<T>(neg ? -x[r].re : x[r].re,
                neg ? -x[r].im : x[r].im);
    }
}

// Gridding: grid (+)= sum of the FFT'd sub-grids covering each cell, in
// the reference's task order (sdp_gridder_subgrid_add, utils.cpp:553-601,
// sequential over tasks), with the sub-grid FFT's output checkerboard, the
// grid IFFT's input checkerboard, and factor (image_size / S)^2. One block
// row per grid row (the sub-grid rows covering it are uniform per block);
// 32-bit index arithmetic (the host checks G < 2^22). The candidate
// sub-grids of a cell (at most kGatherCand per axis, host-checked) are
// collected first, then all their slot lookups and then all their loads
// are issued before the first is used: the kernel is bound by memory
// latency, and a cell's 2-4 sub-grids were read one dependent pair of
// loads at a time.
template<typename T, int kGatherCand>
__global__ void k_gather_grid(Cx<T>* __restrict__ grid, int64_t G64,
        const Cx<T>* __restrict__ stack, int S,
        const int* __restrict__ slot_of, int64_t nu64, int64_t nv64,
        int64_t min_iu64, int64_t min_iv64, int eff, T factor, int accumulate)
{
#pragma clang fp contract(off)
    const int G = (int)G64, nu = (int)nu64, nv = (int)nv64;
    const int min_iu = (int)min_iu64, min_iv = (int)min_iv64;
    const int gv = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int gu = (int)blockIdx.y;
    if (gv >= G) return;
    const int64_t gi = (int64_t)gu * G + gv;
    const float inv_eff = 1.0f / (float)eff;
    // Candidates along each axis, ascending (wrap k = -1, 0, 1, then index).
    int ua[kGatherCand], uu[kGatherCand], vb[kGatherCand], vv[kGatherCand];
    const int nuc = gather_candidates(gu - G / 2 + S / 2, G, S, eff, inv_eff,
            min_iu, nu, ua, uu);
    const int nvc = gather_candidates(gv - G / 2 + S / 2, G, S, eff, inv_eff,
            min_iv, nv, vb, vv);
    constexpr int kC = kGatherCand * kGatherCand;
    int slot[kC];
#pragma unroll
    for (int c = 0; c < kC; ++c)
    {
        const int cu = c / kGatherCand, cv = c % kGatherCand;
        slot[c] = (cu < nuc && cv < nvc) ? slot_of[uu[cu] * nv + vv[cv]] : -1;
    }
    const int64_t SS = (int64_t)S * S;
    Cx<T> x[kC];
#pragma unroll
    for (int c = 0; c < kC; ++c)
    {
        const int cu = c / kGatherCand, cv = c % kGatherCand;
        x[c] = (slot[c] >= 0) ? stack[slot[c] * SS + ua[cu] * S + vb[cv]] :
                cx<T>(0, 0);
    }
    Cx<T> acc = accumulate ? grid[gi] : cx<T>(0, 0);
    const bool neg_g = ((gu + gv) & 1) != 0;
#pragma unroll
    for (int c = 0; c < kC; ++c)
    {
        if (slot[c] < 0) continue;
        const int cu = c / kGatherCand, cv = c % kGatherCand;
        const bool neg = ((ua[cu] + vb[cv]) & 1) != 0;
        T re = (neg ? -x[c].re : x[c].re) * factor;
        T im = (neg ? -x[c].im : x[c].im) * factor;
        if (neg_g)
        {
            re = -re;
            im = -im;
        }
        acc.re += re;
        acc.im += im;
    }
    grid[gi] = acc;
}

// No-wrap form of k_gather_grid, for a plane whose sub-grids all lie inside
// the grid along both axes (host-checked; config 4 and every small test):
// the sub-grids covering cell x are then the k = 0 image's ii in
// [ceil((x - S + 1) / eff), floor(x / eff)], at most NC = ceil(S / eff) per
// axis, ascending -- the same set and order as gather_candidates, so the
// same sums. A thread takes kGatherRows consecutive rows of one column
// (the column's candidates are found once) and issues all their slot
// lookups, then all their sub-grid loads. The general kernel spent ~300
// instructions per cell on the three periodic images' candidate loops
// (SQ counters, config 4); this one ~1/4 of that.
constexpr int kGatherRows = 4;

template<int NC>
__device__ __forceinline__ int gather_candidates_nw(int x, int S, int eff,
        float inv_eff, int lo_idx, int n_idx, int (&off)[NC], int (&idx)[NC])
{
    const int i_lo = max(floor_div_small(x - S + eff, eff, inv_eff), lo_idx);
    const int i_hi = min(floor_div_small(x, eff, inv_eff), lo_idx + n_idx - 1);
    int nc = 0;
#pragma unroll
    for (int k = 0; k < NC; ++k)
    {
        const int ii = i_lo + k;
        off[k] = x - ii * eff;
        idx[k] = ii - lo_idx;
        if (ii <= i_hi) nc = k + 1;
    }
    return nc;
}

template<typename T, int NC>
__global__ void k_gather_grid_nw(Cx<T>* __restrict__ grid, int G,
        const Cx<T>* __restrict__ stack, int S,
        const int* __restrict__ slot_of, int nu, int nv, int min_iu,
        int min_iv, int eff, T factor, int accumulate)
{
#pragma clang fp contract(off)
    const int gv = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int gu0 = (int)blockIdx.y * kGatherRows;
    if (gv >= G) return;
    const float inv_eff = 1.0f / (float)eff;
    int vb[NC], vv[NC];
    const int nvc = gather_candidates_nw(gv - G / 2 + S / 2, S, eff, inv_eff,
            min_iv, nv, vb, vv);
    constexpr int kC = NC * NC;
    const int64_t SS = (int64_t)S * S;
    int ua[kGatherRows][NC];
    int slot[kGatherRows][kC];
#pragma unroll
    for (int r = 0; r < kGatherRows; ++r)
    {
        int uu[NC];
        const int gu = min(gu0 + r, G - 1);
        const int nuc = gather_candidates_nw(gu - G / 2 + S / 2, S, eff,
                inv_eff, min_iu, nu, ua[r], uu);
#pragma unroll
        for (int c = 0; c < kC; ++c)
        {
            const int cu = c / NC, cv = c % NC;
            slot[r][c] = (cu < nuc && cv < nvc && gu0 + r < G) ?
                    slot_of[uu[cu] * nv + vv[cv]] : -1;
        }
    }
    Cx<T> x[kGatherRows][kC];
#pragma unroll
    for (int r = 0; r < kGatherRows; ++r)
#pragma unroll
        for (int c = 0; c < kC; ++c)
        {
            const int cu = c / NC, cv = c % NC;
            x[r][c] = (slot[r][c] >= 0) ?
                    stack[slot[r][c] * SS + ua[r][cu] * S + vb[cv]] :
                    cx<T>(0, 0);
        }
#pragma unroll
    for (int r = 0; r < kGatherRows; ++r)
    {
        const int gu = gu0 + r;
        if (gu >= G) break;
        const int64_t gi = (int64_t)gu * G + gv;
        Cx<T> acc = accumulate ? grid[gi] : cx<T>(0, 0);
        const bool neg_g = ((gu + gv) & 1) != 0;
#pragma unroll
        for (int c = 0; c < kC; ++c)
        {
            if (slot[r][c] < 0) continue;
            const int cu = c / NC, cv = c % NC;
            const bool neg = ((ua[r][cu] + vb[cv]) & 1) != 0;
            T re = (neg ? -x[r][c].re : x[r][c].re) * factor;
            T im = (neg ? -x[r][c].im : x[r][c].im) * factor;
            if (neg_g)
            {
                re = -re;
                im = -im;
            }
            acc.re += re;
            acc.im += im;
        }
        grid[gi] = acc;
    }
}

// Image-side kernels: kImgRows grid rows per thread (blockIdx.y), all rows'
// loads (grid / image values and correction scales) issued before the
// arithmetic: these passes are bound by memory latency.
constexpr int kImgRows = 4;

// Gridding, image side of a w-stack plane: image += grid_correct(
// checkerboard(IFFT(grid)) / G^2) (.cpp:702-711).
template<typename T>
__global__ void k_image_update(const Cx<T>* __restrict__ grid, int64_t G,
        AnyView image, T norm, CorrParams cp, int perm_n2)
{
#pragma clang fp contract(off)
    const int64_t gv = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    // blockIdx.y: kImgRows consecutive rows of the grid as stored; with the
    // fused FFT's permuted rows (perm_n2 > 0), stored row s holds natural
    // row (s % N1) N2 + s / N1, so the grid reads stay consecutive and the
    // image rows of a thread are N2 apart.
    const int64_t s0 = (int64_t)blockIdx.y * kImgRows;
    if (gv >= G) return;
    auto natural = [&](int64_t s) -> int64_t {
        if (!perm_n2) return s;
        const int64_t n1 = G / perm_n2;
        return (s % n1) * perm_n2 + s / n1;
    };
    constexpr int kind = sizeof(T) == 8 ? 3 : 2;
    const int pm = (int)(gv - G / 2);
    Cx<T> x[kImgRows];
    Cx<double> o[kImgRows];
    double sc[kImgRows];
#pragma unroll
    for (int r = 0; r < kImgRows; ++r)
    {
        const int64_t st = s0 + r;
        const bool ok = st < G;
        const int64_t gu = natural(ok ? st : 0);
        x[r] = grid[(ok ? st : 0) * G + gv];
        o[r] = image.load(gu * G + gv);
        const int pl = (int)(gu - G / 2);
        sc[r] = (ok && corr_inside(pl, pm, cp)) ?
                corr_scale(pl, pm, kind, cp) : 1.0;
    }
#pragma unroll
    for (int r = 0; r < kImgRows; ++r)
    {
        if (s0 + r >= G) break;
        const int64_t gu = natural(s0 + r);
        Cx<T> v = x[r];
        if (parity_sign(gu + gv) < 0)
        {
            v.re = -v.re;
            v.im = -v.im;
        }
        v.re *= norm;
        v.im *= norm;
        const int pl = (int)(gu - G / 2);
        Cx<double> z = cx<double>(v.re, v.im);
        if (corr_inside(pl, pm, cp))
            z = (kind == 2) ? correct_scaled_f32(z, pl, pm, cp, (float)sc[r]) :
                    correct_scaled(z, kind, pl, pm, cp, sc[r]);
        Cx<double> out = o[r];
        out.re += z.re;
        if (image.kind >= 2) out.im += z.im;
        image.store(gu * G + gv, out);
    }
}

// Degridding, image side of a w-stack plane: grid = checkerboard(
// degrid_correct((T)image)) ahead of the forward FFT (.cpp:363-375).
template<typename T>
__global__ void k_image_to_grid(AnyView image, int64_t G,
        Cx<T>* __restrict__ grid, CorrParams cp)
{
#pragma clang fp contract(off)
    const int64_t gv = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t gu0 = (int64_t)blockIdx.y * kImgRows;
    if (gv >= G) return;
    constexpr int kind = sizeof(T) == 8 ? 3 : 2;
    const int pm = (int)(gv - G / 2);
    Cx<double> a[kImgRows];
    double sc[kImgRows];
#pragma unroll
    for (int r = 0; r < kImgRows; ++r)
    {
        const int64_t gu = gu0 + r;
        const bool ok = gu < G;
        a[r] = image.load((ok ? gu : 0) * G + gv);
        const int pl = (int)(gu - G / 2);
        sc[r] = (ok && corr_inside(pl, pm, cp)) ?
                corr_scale(pl, pm, kind, cp) : 1.0;
    }
#pragma unroll
    for (int r = 0; r < kImgRows; ++r)
    {
        const int64_t gu = gu0 + r;
        if (gu >= G) break;
        const int pl = (int)(gu - G / 2);
        Cx<double> z = cx<double>((double)(T)a[r].re, (double)(T)a[r].im);
        if (corr_inside(pl, pm, cp))
            z = (kind == 2) ? correct_scaled_f32(z, pl, pm, cp, (float)sc[r]) :
                    correct_scaled(z, kind, pl, pm, cp, sc[r]);
        T re = (T)z.re, im = (T)z.im;
        if (parity_sign(gu + gv) < 0)
        {
            re = -re;
            im = -im;
        }
        grid[gu * G + gv] = cx<T>(re, im);
    }
}

// ---------------------------------------------------------------------------
// Workgroup barrier that first drains this wave's LDS operations. Without
// the explicit lgkmcnt(0), a barrier on a loop back-edge of k_tower_idft
// was reached with an LDS store still in flight and another wave's read
// after the barrier missed it (about 1 in 2000 visibilities lost one
// 16 x 16 block's partial).
__device__ __forceinline__ void lds_sync()
{
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
    __syncthreads();
}

// Fused w-tower gridding for complex-float visibilities (k_tower_dft).
//
// The reference moves a w_support-deep stack of S x S sub-grids through
// every w-layer of a tower with one S x S inverse FFT per layer
// (sdp_gridder_wtower_uvw.cpp:1024-1113). A layer holds only the taps of
// the few visibilities whose w-kernel reaches it, so its inverse FFT is a
// sum of separable outer products: for a visibility with uv taps at rows
// a = iu0 + du and columns b = iv0 + dv,
//   checker(IFFT(layer))[l][m] += kw_j V KU(l) KV(m),
//   KU(l) = sum_du ku[du] E(iu0 + du, l), E(a, l) = (-1)^(a+l) e^{2 pi i a l / S}
// (the checkerboards on both sides of the FFT folded into E). Following
// the recurrence wimg = wimg / D + layer to the end of the tower and the
// final wimg * D^(last + w_support/2 - 1), a visibility gridded at w-layer
// P with w-tap j ends up multiplied by D^(P + j - w_support/2), whatever
// the tower's range. So one workgroup per (sub-grid, 32 x 32
// pixel tile) keeps the sub-grid image in f64 registers for the whole
// tower and, per w-layer L, adds the complex rank-n product
//   M_L = sum_{n : P_n <= L < P_n + w_support} (kw V KU)_n (x) KV_n
// on the matrix core (4 x v_mfma_f32_16x16x4_f32 per 4 visibilities) after
// acc = acc / D (as a multiply by the precomputed 1 / D): the stack, its
// per-layer FFTs and their HBM traffic disappear. Visibilities are staged
// in an LDS ring (their tap sums over the tile's 32 rows and 32 columns,
// in f32 like the reference's complex-float layers); the per-layer window
// comes from an LDS table of layer starts.
// D^e from the phase table, to f32 accuracy: the phase e * turns is reduced
// to [-1/2, 1/2] turns in double and evaluated in single precision. Used
// where the product is rounded to single precision anyway (end of a
// gridding tower, start of a degridding one); binary powering in double
// cost ~50 double operations and a 16-byte load per pixel.
__device__ __forceinline__ Cx<double> pattern_pow_f32(double turns, int e)
{
    const double t = (double)e * turns;
    const float f = (float)(t - rint(t));
    float sn, cs;
    sincospif(2.0f * f, &sn, &cs);
    return cx<double>((double)cs, (double)sn);
}

// Per-visibility staging record of the fused tower kernels, written once
// per call by k_dft_prep instead of being rebuilt by every tile's
// workgroup (which cost three dependent global round trips per staging
// pass: record, uvw, kernel rows): words [0] iu0 (-1: invalid), [1] iv0,
// [2] P (w-layer, tower numbering), [3] unused, [4, 6) V, [6, 8) zero, then
// the W u taps and W v taps (f32, zero if invalid; the u taps start on a
// 16-byte boundary), then 16 w taps keyed by absolute w-layer, (P + j) % 16
// (zeros elsewhere). Records are copied whole into the LDS ring.
constexpr int kPrepHdr = 8;
__host__ __device__ constexpr int prep_stride(int W)
{
    return (kPrepHdr + 2 * W + 16 + 3) & ~3;
}

// Waves per SIMD of the two-block tower kernels: 4 with a few spilled
// dwords measured faster than 3 without (dft 24.6 -> 23.0 ms, idft 34.9 ->
// 33.4 ms per plane at config 4); the LDS (33-35 KB + the S twiddles) fits
// four workgroups per CU.
#ifndef TOWER_DFT_WAVES
#define TOWER_DFT_WAVES 4
#endif
#ifndef TOWER_IDFT_WAVES
#define TOWER_IDFT_WAVES 6
#endif
// k_tower_idft: staged visibilities (ring) and w-layers between re-anchored
// images (see k_tower_idft). 8-wave workgroups of one block per wave (half
// the per-lane pixel state, 6-8 waves per SIMD) measured 20.0 -> 22.4 ms
// (k_tower_dft) and 31.1 -> 35.0 ms (k_tower_idft) per config-4 plane and
// were removed.
constexpr int kIdftCap = 16;
constexpr int kIdftBlock = 16;
constexpr int kDftCap = 32;      // staged visibilities (ring)
constexpr int kDftTile = 32;     // tile edge (pixels)
constexpr int kDftLayers = 512;  // max w-layers of a sub-grid's tower
constexpr int kDftMaxS = 1024;
constexpr int kDftBlock = 8;     // w-layers per f32 recurrence block
static_assert((kDftCap & (kDftCap - 1)) == 0 && (kDftTile & (kDftTile - 1)) == 0,
        "ring slots and tile offsets are taken with masks");

struct DftParams
{
    TowerParams tp;                 // group's tower parameters
    const int4* vrec;               // row, channel, layer (rel. P0), gslot
    const int* seg_start;           // [gslot] first visibility
    const int* seg_end;             // [gslot] end
    int64_t gslot_base;             // group * t_cap
    int64_t P0;
    Cx<float>* out;                 // [slots][S][S] (stack layer 0)
    const Cx<double>* wp;           // D
    const Cx<double>* wp_inv;       // 1 / D
    const double* w_turns;          // D = exp(2 pi i w_turns)
    const double* uv_kernel;
    const double* w_kernel;
    const float2* tw;               // e^{2 pi i k / S}, k < S
    const float* prep;              // per-visibility staging records
    int prep_stride;                // words per record (prep_stride(W))
    float norm;                     // degrid: 1 / S^2 of the sub-grid IFFT
    const Cx<float>* in;            // degrid: [slots][S][S] sub-grid images
    float2* part;                   // degrid: [visibility][tile] partials
};

// Tap DFT of a visibility's W kernel taps at one tile row / column:
// sum_du kt[du] e^{2 pi i (idx + du step) / S} (checkerboard folded into
// idx and step by the callers): Horner in z = e^{2 pi i step / S}, then one
// product with e^{2 pi i idx / S} -- two twiddle-table reads instead of W
// (the per-tap table form: the rows the lanes of a wave read are (a0 + du)
// l apart, ~3.5-way LDS bank conflicts; 23.3 -> 21.9 ms per plane).
// f32 rounding of the recurrence: ~W ulp.

__device__ __forceinline__ float2 tap_dft(const float* kt, int W,
        const float2* s_tw, int idx, int step, int S)
{
#pragma clang fp contract(off)
    const float2 z = s_tw[step], e0 = s_tw[idx];
    float ar = kt[W - 1], ai = 0.0f;
    for (int du = W - 2; du >= 0; --du)
    {
        const float nr = __builtin_fmaf(ar, z.x,
                __builtin_fmaf(-ai, z.y, kt[du]));
        const float ni = __builtin_fmaf(ar, z.y, ai * z.x);
        ar = nr;
        ai = ni;
    }
    return make_float2(__builtin_fmaf(ar, e0.x, -(ai * e0.y)),
            __builtin_fmaf(ar, e0.y, ai * e0.x));
}

// Same, W known at compile time (the common W = 8): the tap reads are
// 16-byte aligned rows (kPrepHdr = 8) and the loop is unrolled.
template<int WT>
__device__ __forceinline__ float2 tap_dft_w(const float* kt,
        const float2* s_tw, int idx, int step)
{
#pragma clang fp contract(off)
    const float* k = static_cast<const float*>(__builtin_assume_aligned(kt, 16));
    const float2 z = s_tw[step], e0 = s_tw[idx];
    float ar = k[WT - 1], ai = 0.0f;
#pragma unroll
    for (int du = WT - 2; du >= 0; --du)
    {
        const float nr = __builtin_fmaf(ar, z.x, __builtin_fmaf(-ai, z.y, k[du]));
        const float ni = __builtin_fmaf(ar, z.y, ai * z.x);
        ar = nr;
        ai = ni;
    }
    return make_float2(__builtin_fmaf(ar, e0.x, -(ai * e0.y)),
            __builtin_fmaf(ar, e0.y, ai * e0.x));
}

__device__ __forceinline__ float2 tap_dft_any(const float* kt, int W,
        const float2* s_tw, int idx, int step, int S)
{
    if (W == 8) return tap_dft_w<8>(kt, s_tw, idx, step);
    return tap_dft(kt, W, s_tw, idx, step, S);
}

// Staged records in LDS: ring slot rs holds visibility record words
// [0, prep_stride) (layout above) at a pitch of 60 words = 4 x 15, so that
// the 16 different slots a quarter-wave reads at one word offset fall on
// 16 different banks.
constexpr int kRecPitch = 60;
static_assert(prep_stride(16) <= kRecPitch, "records of W <= 16 fit a slot");

// Ring slots (x .. x + cnt) & (CAP - 1) <- records v0 .. v0 + cnt - 1:
// 16-byte copies, 16 threads per record (no per-word branches).
template<int CAP, int NT = 256>
__device__ __forceinline__ void stage_records(const DftParams& d, int64_t v0,
        int x, int cnt, int t, float (*s_rec)[kRecPitch])
{
    const int nq = d.prep_stride / 4;
    const float4* src = reinterpret_cast<const float4*>(d.prep +
            v0 * d.prep_stride);
    for (int o = t; o < cnt * 16; o += NT)
    {
        const int vi = o >> 4, k = o & 15;
        if (k < nq)
            *reinterpret_cast<float4*>(&s_rec[(x + vi) & (CAP - 1)][4 * k]) =
                    src[vi * nq + k];
    }
}

// NB: 16 x 16 pixel blocks per wave along the columns. A workgroup owns a
// 32 x (32 NB) pixel tile; with NB = 2 each wave's two blocks share the row
// taps (A operand) and the per-layer window / Horner bookkeeping, and their
// independent accumulation chains keep the matrix core busier.
template<typename U, int NB, int NW = 4>
__global__ __launch_bounds__(64 * NW)
__attribute__((amdgpu_waves_per_eu(NB == 2 ? TOWER_DFT_WAVES : 1)))
void k_tower_dft(
        DftParams d,
        const U* __restrict__ uvws, const Cx<float>* __restrict__ vis)
{
#pragma clang fp contract(off)
    // NW waves: NW / 2 per 16-row block band, NB 16 x 16 blocks each.
    constexpr int NT = 64 * NW, kCW = NW / 2;
    constexpr int kNbOff = 16 * kCW;                 // column step of nb
    constexpr int kCols = kNbOff * NB;               // tile columns
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    extern __shared__ float2 s_tw[];                // e^{2 pi i k / S}, S
    __shared__ int s_start[kDftLayers + 1];
    __shared__ float2 s_aku[kDftCap][kDftTile];     // V KU(l), tile rows
    __shared__ float2 s_kv[kDftCap][kCols];         // KV(m), tile columns
    // Staged records: iu0 (-1: invalid), iv0, V, u taps, v taps, and the
    // w taps keyed by absolute w-layer, word kwo + (P + j) % 16 = kw_j, so
    // the rank update reads kw at layer L without first reading P.
    __shared__ __attribute__((aligned(16))) float s_rec[kDftCap][kRecPitch];

    const TowerParams& tp = d.tp;
    const int S = tp.S, ws = tp.w_support, W = tp.support;
    const int kwo = kPrepHdr + 2 * W;   // w taps in a staged record
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int tiles_v = S / kCols;
    const int L0 = (blockIdx.x / tiles_v) * kDftTile;
    const int M0 = (blockIdx.x % tiles_v) * kCols;
    const int slot = blockIdx.y;
    const int64_t gs = d.gslot_base + slot;
    const int s0 = d.seg_start[gs], s1 = d.seg_end[gs];
    const int n = s1 - s0;
    // This lane's pixels: block (wave / kCW, wave % kCW) of the tile, MFMA
    // C layout: rows 4 (lane >> 4) + r, column lane & 15.
    const int bl = (wave / kCW) * 16, bm = (wave % kCW) * 16;
    const int i = lane & 15, kq = lane >> 4;
    const int pm = M0 + bm + i;       // column of block 0; block nb: + kNbOff nb
    // The recurrence wimg = wimg / D + M_L runs in f32 within blocks of
    // kDftBlock layers (acc32, 1 / D rounded to f32) and in f64 across
    // blocks (acc64 = acc64 / D^kDftBlock + acc32): the reference keeps
    // wimg in complex double; the block partial sums carry the f32
    // rounding of kDftBlock steps, like its complex-float layers.
    // The f32 block partial lives in the matrix-core accumulators: each
    // layer first scales it by 1 / D, then the layer's rank update is
    // accumulated onto it (no zeroing / read-back of a separate layer sum).
    Cx<double> acc[NB][4], dinv_k[NB][4];
    float2 dinv32[NB][4];
    f32x4 a_re[NB], a_im[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
    {
        a_re[nb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        a_im[nb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const int64_t e = (int64_t)(L0 + bl + 4 * kq + r) * S + pm +
                    kNbOff * nb;
            acc[nb][r] = cx<double>(0.0, 0.0);
            const Cx<double> di = d.wp_inv[e];
            dinv32[nb][r] = make_float2((float)di.re, (float)di.im);
            dinv_k[nb][r] = cpow_int(di, kDftBlock);
        }
    }
    Cx<float>* out = d.out + (int64_t)slot * S * S;
    if (n <= 0)
    {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                out[(int64_t)(L0 + bl + 4 * kq + r) * S + pm + kNbOff * nb] =
                        cx<float>(0, 0);
        return;
    }
    for (int k = t; k < S; k += NT) s_tw[k] = d.tw[k];
    // Layer starts: s_start[k] = first visibility with P >= P_first + k.
    // w-layers in the tower's numbering (TowerParams::w_plane).
    const int shift = (int)(d.P0 - tp.off_w);
    const int P_first = d.vrec[s0].z + shift, P_last = d.vrec[s1 - 1].z + shift;
    const int npl = P_last - P_first + 1;
    if (t == 0)
    {
        s_start[0] = 0;
        s_start[npl] = n;
    }
    for (int v = t + 1; v < n; v += NT)
    {
        const int pa = d.vrec[s0 + v - 1].z + shift - P_first;
        const int pb = d.vrec[s0 + v].z + shift - P_first;
        for (int k = pa + 1; k <= pb; ++k) s_start[k] = v;
    }
    int st_lo = 0, st_hi = 0;     // staged range (uniform)
    lds_sync();

    const int L_first = P_first, L_last = P_last + ws - 1;
    // Blocks end at L_last: the first block takes the remainder.
    const int n_layers = L_last - L_first + 1;
    const int blk_off = (kDftBlock - n_layers % kDftBlock) % kDftBlock;
    for (int L = L_first; L <= L_last; ++L)
    {
        const int lo = s_start[max(0, min(npl, L - ws + 1 - P_first))];
        const int hi = s_start[max(0, min(npl, L + 1 - P_first))];
        // wimg = wimg / D (f32 within the block), then + layer below.
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                const float xr = a_re[nb][r], xi = a_im[nb][r];
                const float2 q = dinv32[nb][r];
                // One rounding fewer than mul + add, and no pair packing.
                a_re[nb][r] = __builtin_fmaf(xr, q.x, -(xi * q.y));
                a_im[nb][r] = __builtin_fmaf(xr, q.y, xi * q.x);
            }
        for (int a = lo; a < hi; a += kDftCap)
        {
            const int b = min(hi, a + kDftCap);
            if (!(a >= st_lo && b <= st_hi))
            {
                // Stage ahead: fill the ring with [a, a + kDftCap), keeping
                // what is already there (windows only move forward, so a
                // staging pass serves the next few w-layers; each pass
                // costs several dependent global round trips).
                const int e = min(n, a + kDftCap);
                const int x = (a >= st_lo && a <= st_hi) ? st_hi : a;
                st_lo = a;
                st_hi = e;
                const int cnt = e - x;
                lds_sync();   // ring slots free
                // Copy the staged visibilities' records (one dependent
                // global load per word, 16-byte coalesced) into the ring.
                stage_records<kDftCap, NT>(d, s0 + x, x, cnt, t, s_rec);
                lds_sync();
                constexpr int kPer = kDftTile + kCols;   // rows, columns
                for (int o = t; o < cnt * kPer; o += NT)
                {
                    const int v = x + (int)((unsigned)o / kPer);
                    const int rs = v & (kDftCap - 1);
                    const int q = (int)((unsigned)o % kPer);
                    const int iu0 = __float_as_int(s_rec[rs][0]);
                    float2 res = make_float2(0.0f, 0.0f);
                    if (iu0 >= 0)
                    {
                        const bool row = q < kDftTile;
                        const int a0 = row ? iu0 : __float_as_int(s_rec[rs][1]);
                        const float* kt = &s_rec[rs][kPrepHdr] + (row ? 0 : W);
                        const int l = row ? L0 + q : M0 + q - kDftTile;
                        // (-1)^(a + l) e^{2 pi i a l / S} = e^{2 pi i k / S}
                        // with k = a l + (a + l) S / 2 (mod S; S is even):
                        // for a = a0, a0 + 1, ... the table index advances
                        // by l + S / 2 per tap, the checkerboard included.
                        const uint32_t us = (uint32_t)S;   // a0, l < S
                        const int idx = (int)(((uint32_t)(a0 * l) +
                                (uint32_t)((a0 + l) & 1) * (us / 2)) % us);
                        const int step = (int)(((uint32_t)l + us / 2) % us);
                        const float2 sv = tap_dft_any(kt, W, s_tw, idx, step, S);
                        const float sr = sv.x, si = sv.y;
                        if (row)
                        {
                            const float2 vv = *reinterpret_cast<const float2*>(
                                    &s_rec[rs][4]);
                            res = make_float2(vv.x * sr - vv.y * si,
                                    vv.x * si + vv.y * sr);
                        }
                        else
                        {
                            res = make_float2(sr, si);
                        }
                    }
                    if (q < kDftTile) s_aku[rs][q] = res;
                    else s_kv[rs][q - kDftTile] = res;
                }
                lds_sync();
            }
            // Complex rank-(b - a) update, four visibilities per step.
            for (int c4 = a; c4 < b; c4 += 4)
            {
                const int v = c4 + kq;
                const bool ok = v < b;
                const int rs = (ok ? v : a) & (kDftCap - 1);
                const float2 av = s_aku[rs][bl + i];
                // Unconditional read + select: no exec-mask branch per step.
                const float kw_rs = s_rec[rs][kwo + (L & 15)];
                const float kw = ok ? kw_rs : 0.0f;
                const float ar = av.x * kw, ai = av.y * kw;
#pragma unroll
                for (int nb = 0; nb < NB; ++nb)
                {
                    const float2 bv = s_kv[rs][bm + kNbOff * nb + i];
                    a_re[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(ar, bv.x,
                            a_re[nb], 0, 0, 0);
                    a_re[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(-ai, bv.y,
                            a_re[nb], 0, 0, 0);
                    a_im[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(ar, bv.y,
                            a_im[nb], 0, 0, 0);
                    a_im[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(ai, bv.x,
                            a_im[nb], 0, 0, 0);
                }
            }
        }
        if ((L - L_first + 1 + blk_off) % kDftBlock == 0)
        {
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
            {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                {
                    Cx<double> z = cmul(acc[nb][r], dinv_k[nb][r]);
                    z.re += (double)a_re[nb][r];
                    z.im += (double)a_im[nb][r];
                    acc[nb][r] = z;
                }
                a_re[nb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
                a_im[nb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            }
        }
    }
    // End of tower: wimg * D^(L_last - w_support / 2) (.cpp:1102-1113),
    // with the checkerboard of the forward FFT that follows.
    const int e_final = L_last - ws / 2;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const int pl = L0 + bl + 4 * kq + r, pc = pm + kNbOff * nb;
            const int64_t e = (int64_t)pl * S + pc;
            Cx<double> z = acc[nb][r];
            if (e_final != 0) z = cmul(z, pattern_pow_f32(d.w_turns[e], e_final));
            float re = (float)z.re, im = (float)z.im;
            if ((pl + pc) & 1)
            {
                re = -re;
                im = -im;
            }
            out[e] = cx<float>(re, im);
        }
}

// Fused w-tower degridding for complex-float visibilities (k_tower_idft),
// the adjoint of k_tower_dft. The reference fills a w_support-deep stack
// with forward FFTs of wimg / D^k and reads each visibility's taps from it
// (sdp_gridder_wtower_uvw.cpp:726-909); with X the sub-grid image after
// the inverse FFT of its cut-out, a visibility gridded at w-layer P reads
//   vis += sum_j kw_j sum_{l,m} X[l][m] D^-(P + j - w_support/2)[l][m]
//          conj(KU)(l) conj(KV)(m)
// (KU, KV as in k_tower_dft). One workgroup per (sub-grid, 32 x 32 pixel
// tile) keeps Y_L = X D^-(L - w_support/2) in registers (f32 within
// kDftBlock layers, re-anchored from f64 across blocks) and, per w-layer,
// forms T = Y_L conj(KV) for 16 visibilities on the matrix core
// (16 x v_mfma_f32_16x16x4_f32 per 16 x 16 pixel block), contracts T with
// conj(KU) on the lanes and accumulates kw-weighted partials per
// visibility in LDS. Partials of a (visibility, tile) pair are added to a
// scratch row owned by the workgroup; k_idft_reduce sums the rows.
// NB: 16 x 16 pixel blocks per wave along the columns (tile 32 x 32 NB);
// with NB = 2 a wave's two blocks extend the contraction T = Y conj(KV) over
// 32 columns before the one row contraction / partial update per chunk.
template<typename U, int NB, int NW = 4>
__global__ __launch_bounds__(64 * NW)
__attribute__((amdgpu_waves_per_eu(NB == 2 ? TOWER_IDFT_WAVES : 1)))
void k_tower_idft(
        DftParams d, const U* __restrict__ uvws)
{
#pragma clang fp contract(off)
    // NW waves: NW / 2 per 16-row block band, NB 16 x 16 blocks each.
    constexpr int NT = 64 * NW, kCW = NW / 2;
    constexpr int kNbOff = 16 * kCW;                 // column step of nb
    constexpr int kCols = kNbOff * NB;               // tile columns
    constexpr int kCap = kIdftCap, kBlk = kIdftBlock;
    static_assert((kCap & (kCap - 1)) == 0 && kCap >= 16, "ring of >= 16");
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    extern __shared__ float2 s_tw[];                // e^{2 pi i k / S}, S
    __shared__ int s_start[kDftLayers + 1];
    // Rows padded by 2 float2: a lane reads 4 consecutive entries of its
    // visibility's row (two 16-byte LDS reads) and the 16 lanes of a
    // quarter-wave, on 16 different rows, then cover all 64 banks once.
    __shared__ float2 s_ku[kCap][kDftTile + 2];  // conj KU(l), tile rows
    __shared__ float2 s_kv[kCap][kCols + 2];     // conj KV(m), tile cols
    __shared__ __attribute__((aligned(16))) float s_rec[kCap][kRecPitch];
    __shared__ float2 s_acc[NW][kCap];           // per-wave partials

    const TowerParams& tp = d.tp;
    const int S = tp.S, ws = tp.w_support, W = tp.support;
    const int kwo = kPrepHdr + 2 * W;   // w taps in a staged record
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int tiles_v = S / kCols;
    const int tile = blockIdx.x;
    const int L0 = (tile / tiles_v) * kDftTile;
    const int M0 = (tile % tiles_v) * kCols;
    const int slot = blockIdx.y;
    const int64_t gs = d.gslot_base + slot;
    const int s0 = d.seg_start[gs], s1 = d.seg_end[gs];
    const int n = s1 - s0;
    if (n <= 0) return;
    const int ntiles = (S / kDftTile) * tiles_v;
    const int bl = (wave / kCW) * 16, bm = (wave % kCW) * 16;
    const int i = lane & 15, kq = lane >> 4;
    const int shift = (int)(d.P0 - tp.off_w);
    const int P_first = d.vrec[s0].z + shift, P_last = d.vrec[s1 - 1].z + shift;
    const int npl = P_last - P_first + 1;
    const int L_first = P_first, L_last = P_last + ws - 1;

    // A-operand pixels of this lane: row bl + i, columns bm + 4 kq + kk
    // (MFMA kk takes its k = kq from column bm + 4 kq + kk; any bijection
    // of the 16 columns works as long as A and B share it, and this one
    // puts a lane's 4 B entries next to each other in LDS).
    // Y_L = X D^-(L - w_support/2) is evaluated afresh from the sub-grid
    // image every kBlk layers (anchor: X in double times the f32-accurate
    // phase, as the reference's complex-double wimg to f32 accuracy) and
    // carried in between by the f32 recurrence Y_{L+1} = Y_L / D (1 / D
    // rounded to f32): no per-pixel double state stays in registers.
    float2 y32[NB][4], dinv32[NB][4];
    const Cx<float>* X = d.in + (int64_t)slot * S * S;
    auto anchor = [&](int L) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
            {
                const int pr = L0 + bl + i;
                const int pc = M0 + kNbOff * nb + bm + 4 * kq + kk;
                const int64_t e = (int64_t)pr * S + pc;
                // Input checkerboard and 1 / S^2 of the sub-grid inverse
                // FFT (.cpp:423-427), in single precision as the reference's
                // layers.
                Cx<float> x = X[e];
                if ((pr + pc) & 1)
                {
                    x.re = -x.re;
                    x.im = -x.im;
                }
                x.re *= d.norm;
                x.im *= d.norm;
                const Cx<double> y = cmul(cx<double>((double)x.re,
                        (double)x.im), pattern_pow_f32(d.w_turns[e],
                        -(L - ws / 2)));
                y32[nb][kk] = make_float2((float)y.re, (float)y.im);
            }
    };
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
        {
            const int pr = L0 + bl + i;
            const int pc = M0 + kNbOff * nb + bm + 4 * kq + kk;
            const Cx<double> di = d.wp_inv[(int64_t)pr * S + pc];
            dinv32[nb][kk] = make_float2((float)di.re, (float)di.im);
        }
    anchor(L_first);
    for (int k = t; k < S; k += NT) s_tw[k] = d.tw[k];
    for (int k = t; k < NW * kCap; k += NT)
        s_acc[k / kCap][k & (kCap - 1)] = make_float2(0.0f, 0.0f);
    if (t == 0)
    {
        s_start[0] = 0;
        s_start[npl] = n;
    }
    for (int v = t + 1; v < n; v += NT)
    {
        const int pa = d.vrec[s0 + v - 1].z + shift - P_first;
        const int pb = d.vrec[s0 + v].z + shift - P_first;
        for (int k = pa + 1; k <= pb; ++k) s_start[k] = v;
    }
    int st_lo = 0, st_hi = 0;
    lds_sync();

    // Adds the partials of staged visibilities [f0, f1) to their scratch
    // rows and clears them (call between barriers). Visibility v is always
    // flushed by thread v % NT, so a scratch entry's read-modify-writes
    // stay in one thread's program order. A visibility is flushed again
    // only when a window wider than the ring re-stages it; below fl_hi
    // (the end of everything flushed so far) the entry is added to, above
    // it stored (the scratch rows start zeroed either way).
    int fl_hi = 0;
    auto flush = [&](int f0, int f1) {
        for (int v = f0 + ((t - f0) % NT + NT) % NT; v < f1; v += NT)
        {
            const int rs = v & (kCap - 1);
            float2 sum = make_float2(0.0f, 0.0f);
#pragma unroll
            for (int w = 0; w < NW; ++w)
            {
                sum.x += s_acc[w][rs].x;
                sum.y += s_acc[w][rs].y;
                s_acc[w][rs] = make_float2(0.0f, 0.0f);
            }
            float2* dst = d.part + (int64_t)(s0 + v) * ntiles + tile;
            if (v < fl_hi)
            {
                const float2 old = *dst;
                sum = make_float2(old.x + sum.x, old.y + sum.y);
            }
            *dst = sum;
        }
        fl_hi = max(fl_hi, f1);
    };

    for (int L = L_first; L <= L_last; ++L)
    {
        const int lo = s_start[max(0, min(npl, L - ws + 1 - P_first))];
        const int hi = s_start[max(0, min(npl, L + 1 - P_first))];
        for (int a = lo; a < hi; a += kCap)
        {
            const int b = min(hi, a + kCap);
            if (!(a >= st_lo && b <= st_hi))
            {
                const int e = min(n, a + kCap);
                const bool keep = a >= st_lo && a <= st_hi;
                const int x = keep ? st_hi : a;
                lds_sync();   // all partials of the ring written
                if (keep) flush(st_lo, a);
                else flush(st_lo, st_hi);
                st_lo = a;
                st_hi = e;
                const int cnt = e - x;
                stage_records<kCap, NT>(d, s0 + x, x, cnt, t, s_rec);
                lds_sync();
                constexpr int kPer = kDftTile + kCols;   // rows, columns
                for (int o = t; o < cnt * kPer; o += NT)
                {
                    const int v = x + (int)((unsigned)o / kPer);
                    const int rs = v & (kCap - 1);
                    const int q = (int)((unsigned)o % kPer);
                    const int iu0 = __float_as_int(s_rec[rs][0]);
                    float2 res = make_float2(0.0f, 0.0f);
                    if (iu0 >= 0)
                    {
                        const bool row = q < kDftTile;
                        const int a0 = row ? iu0 : __float_as_int(s_rec[rs][1]);
                        const float* kt = &s_rec[rs][kPrepHdr] + (row ? 0 : W);
                        const int l = row ? L0 + q : M0 + q - kDftTile;
                        // Checkerboard folded into the index as in
                        // k_tower_dft.
                        const uint32_t us = (uint32_t)S;   // a0, l < S
                        const int idx = (int)(((uint32_t)(a0 * l) +
                                (uint32_t)((a0 + l) & 1) * (us / 2)) % us);
                        const int step = (int)(((uint32_t)l + us / 2) % us);
                        const float2 sv = tap_dft_any(kt, W, s_tw, idx, step, S);
                        res = make_float2(sv.x, -sv.y);   // conjugate
                    }
                    if (q < kDftTile) s_ku[rs][q] = res;
                    else s_kv[rs][q - kDftTile] = res;
                }
                lds_sync();
            }
            // 16 visibilities per step: T = Y_L conj(KV) on the matrix core.
            for (int c16 = a; c16 < b; c16 += 16)
            {
                const int v = c16 + i;
                const bool ok = v < b;
                // Column i of T only sees column i of B: a lane past the
                // window reads a staged row and its result is dropped below.
                const int rs = (ok ? v : a) & (kCap - 1);
                // Complex product in three real matrix products (Gauss):
                // t1 = Yr Kr, t2 = Yi Ki, t3 = (Yr + Yi)(Kr + Ki), then
                // T = (t1 - t2) + i (t3 - t1 - t2): 3 instead of 4 matrix
                // ops per column group (the matrix core is the busiest
                // unit here: a chunk is 16 visibilities wide, a w-layer's
                // window holds ~5).
                f32x4 t1 = {0.0f, 0.0f, 0.0f, 0.0f};
                f32x4 t2 = {0.0f, 0.0f, 0.0f, 0.0f};
                f32x4 t3 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int nb = 0; nb < NB; ++nb)
                {
                    float2 bv[4];
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk)
                        bv[kk] = s_kv[rs][kNbOff * nb + bm + 4 * kq + kk];
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk)
                    {
                        const float yr = y32[nb][kk].x, yi = y32[nb][kk].y;
                        t1 = __builtin_amdgcn_mfma_f32_16x16x4f32(yr,
                                bv[kk].x, t1, 0, 0, 0);
                        t2 = __builtin_amdgcn_mfma_f32_16x16x4f32(yi,
                                bv[kk].y, t2, 0, 0, 0);
                        t3 = __builtin_amdgcn_mfma_f32_16x16x4f32(yr + yi,
                                bv[kk].x + bv[kk].y, t3, 0, 0, 0);
                    }
                }
                f32x4 t_re, t_im;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                {
                    t_re[r] = t1[r] - t2[r];
                    t_im[r] = t3[r] - t1[r] - t2[r];
                }
                // Rows 4 kq + r of T for visibility i: contract with conj KU.
                float pr = 0.0f, pi = 0.0f;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                {
                    const float2 ku = s_ku[rs][bl + 4 * kq + r];
                    pr = __builtin_fmaf(ku.x, t_re[r], pr);
                    pr = __builtin_fmaf(-ku.y, t_im[r], pr);
                    pi = __builtin_fmaf(ku.x, t_im[r], pi);
                    pi = __builtin_fmaf(ku.y, t_re[r], pi);
                }
                pr = sdp_hip::sum_rows16(pr);
                pi = sdp_hip::sum_rows16(pi);
                if (kq == 0 && ok)
                {
                    const float kw = s_rec[rs][kwo + (L & 15)];
                    float2 acc = s_acc[wave][rs];
                    acc.x += pr * kw;
                    acc.y += pi * kw;
                    s_acc[wave][rs] = acc;
                }
            }
        }
        // Y_{L+1} = Y_L / D.
        if ((L + 1 - L_first) % kBlk == 0)
        {
            if (L < L_last) anchor(L + 1);
        }
        else
        {
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                {
                    const float2 yv = y32[nb][kk], q = dinv32[nb][kk];
                    y32[nb][kk] = make_float2(
                            __builtin_fmaf(yv.x, q.x, -(yv.y * q.y)),
                            __builtin_fmaf(yv.x, q.y, yv.y * q.x));
                }
        }
    }
    lds_sync();
    flush(st_lo, st_hi);
}

// vis[row, channel] += sum over the tiles of the scratch row.
__global__ void k_idft_reduce(const int4* __restrict__ vrec, int64_t n_vis,
        const float2* __restrict__ part, int ntiles, int64_t num_chan,
        Cx<float>* __restrict__ vis)
{
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= n_vis) return;
    const float2* p = part + v * ntiles;
    float sr = 0.0f, si = 0.0f;
    for (int k = 0; k < ntiles; ++k)
    {
        const float2 x = p[k];
        sr += x.x;
        si += x.y;
    }
    const int4 rec = vrec[v];
    Cx<float>* out = vis + (int64_t)rec.x * num_chan + rec.y;
    atomicAdd(&out->re, sr);
    atomicAdd(&out->im, si);
}

__global__ void k_twiddles(float2* __restrict__ tw, int S)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= S) return;
    double sn, cs;
    sincospi(2.0 * k / S, &sn, &cs);
    tw[k] = make_float2((float)cs, (float)sn);
}

__global__ void k_pattern_inv(const Cx<double>* __restrict__ wp,
        Cx<double>* __restrict__ inv, int64_t n)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) inv[i] = cdiv(cx<double>(1.0, 0.0), wp[i]);
}

// Phase of the w-pattern in turns, w_step n(l, m) (D = exp(2 pi i turns),
// sdp_gridder_utils.cpp:1353-1380; the host table's pixel geometry).
__global__ void k_pattern_turns(double* __restrict__ turns, int S,
        double theta, double shear_u, double shear_v, double w_step)
{
#pragma clang fp contract(off)
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= (int64_t)S * S) return;
    const int il = (int)(i / S), im = (int)(i % S);
    const double l = (il - S / 2) * theta / S;
    const double m = (im - S / 2) * theta / S;
    turns[i] = w_step * lm_to_n_dev(l, m, shear_u, shear_v);
}


// Expand sorted visibility runs (row, c0, c1, slot) into one record per
// channel: (row, channel, w-layer relative to P0, group slot id).
__global__ void k_expand_runs(const int4* __restrict__ items,
        const uint64_t* __restrict__ keys, const int64_t* __restrict__ off,
        int64_t n_items, int64_t NP, int4* __restrict__ vrec)
{
    const int64_t it = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (it >= n_items) return;
    const int4 r = items[it];
    const uint64_t key = keys[it];
    const int p_rel = (int)(key % (uint64_t)NP);
    const int gslot = (int)(key / (uint64_t)NP);
    int64_t o = off[it];
    for (int c = r.y; c < r.z; ++c) vrec[o++] = make_int4(r.x, c, p_rel, gslot);
}

__global__ void k_run_channels(const int4* __restrict__ items, int64_t n,
        int64_t* __restrict__ cnt)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) cnt[i] = items[i].z - items[i].y;
}

__global__ void k_segments(const int4* __restrict__ vrec, int64_t n,
        int* __restrict__ seg_start, int* __restrict__ seg_end)
{
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= n) return;
    const int gs = vrec[v].w;
    if (v == 0 || vrec[v - 1].w != gs) seg_start[gs] = (int)v;
    if (v == n - 1 || vrec[v + 1].w != gs) seg_end[gs] = (int)(v + 1);
}

// Per-visibility staging records (see prep_stride), and a flag for
// visibilities whose uv taps leave the sub-grid: the reference wraps them
// through its flat [w_support][S][S] stack indexing, which only the
// layer-by-layer path reproduces.
template<typename U>
__global__ void k_dft_prep(const int4* __restrict__ vrec, int64_t n,
        const U* __restrict__ uvws, const Cx<float>* __restrict__ vis,
        TowerParams base, const int* __restrict__ tasks,
        const int* __restrict__ g_offw, const int* __restrict__ g_tbase,
        int64_t t_cap, int64_t P0, const double* __restrict__ uv_kernel,
        const double* __restrict__ w_kernel, float* __restrict__ prep,
        int* __restrict__ flag)
{
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= n) return;
    const int4 rec = vrec[v];
    const int group = (int)(rec.w / t_cap), slot = (int)(rec.w % t_cap);
    TowerParams q = base;
    q.off_w = g_offw[group];
    q.w_plane = (int)(rec.z + P0 - q.off_w);
    const int task = tasks[g_tbase[group] + slot];
    const int off_u = (int)((q.min_iu + task / q.nv) * q.eff);
    const int off_v = (int)((q.min_iv + task % q.nv) * q.eff);
    const Taps2 tt = item_taps(q, uvws, rec.x, rec.y, off_u, off_v);
    if (tt.valid && (tt.iu0 < 0 || tt.iu0 + q.support > q.S ||
            tt.iv0 < 0 || tt.iv0 + q.support > q.S))
        atomicOr(flag, 1);
    const int W = q.support, ws = q.w_support;
    float* r = prep + v * prep_stride(W);
    r[0] = __int_as_float(tt.valid ? tt.iu0 : -1);
    r[1] = __int_as_float(tt.iv0);
    r[2] = __int_as_float(q.w_plane);
    r[3] = 0.0f;
    float vre = 0.0f, vim = 0.0f;
    if (vis)
    {
        const Cx<float> vv = vis[(int64_t)rec.x * q.num_chan + rec.y];
        vre = vv.re;
        vim = vv.im;
    }
    r[4] = vre;
    r[5] = vim;
    r[6] = 0.0f;
    r[7] = 0.0f;
    for (int j = 0; j < W; ++j)
    {
        r[kPrepHdr + j] = tt.valid ? (float)uv_kernel[tt.u_off + j] : 0.0f;
        r[kPrepHdr + W + j] = tt.valid ? (float)uv_kernel[tt.v_off + j] : 0.0f;
    }
    float kw[16];
    for (int k = 0; k < 16; ++k) kw[k] = 0.0f;
    for (int j = 0; j < ws; ++j)
        kw[(q.w_plane + j) & 15] = tt.valid ? (float)w_kernel[tt.w_off + j] :
                0.0f;
    for (int k = 0; k < 16; ++k) r[kPrepHdr + 2 * W + k] = kw[k];
    for (int k = kPrepHdr + 2 * W + 16; k < prep_stride(W); ++k) r[k] = 0.0f;
}

// Per-pixel correction scale of a plan's facet, 1 / (pswf(l) pswf(m)
// pswf_n(n)) -- a geometric constant: every w-stack plane's correction
// multiplies by the same value, so the image-side kernels read it (4 bytes
// per pixel for float facets) instead of evaluating the PSWFs per call.
template<typename S>
__global__ void k_scale_table(CorrParams cp, S* __restrict__ tab)
{
    const int64_t im = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t il = blockIdx.y;
    const int N = cp.image_size;
    if (im >= N) return;
    tab[il * N + im] = (S)pixel_scale((int)il - N / 2, (int)im - N / 2, cp);
}

// ---------------------------------------------------------------------------
// Host side.

unsigned blocks_of(int64_t n, int t = 256)
{
    return (unsigned)((n + t - 1) / t);
}

// Device buffers reused across calls (grown on demand).
struct Workspace
{
    std::vector<std::pair<void*, size_t> > buf;

    void* get(size_t id, size_t bytes, sdp_Error* status)
    {
        if (buf.size() <= id) buf.resize(id + 1, {nullptr, 0});
        if (buf[id].second < bytes)
        {
            if (buf[id].first) (void)hipFree(buf[id].first);
            buf[id] = {nullptr, 0};
            SDP_HIP_CHECK(hipMalloc(&buf[id].first, bytes), status);
            if (*status) return nullptr;
            buf[id].second = bytes;
        }
        return buf[id].first;
    }
};

enum BufId
{
    kRowCount, kRowOffset, kOccupied, kSlotMap, kKeys, kKeysAlt, kIdx,
    kIdxAlt, kItemsRaw, kItems, kHist, kTemp, kTasks, kSlotOf, kBounds,
    kStack, kWimg, kGrid, kVrec, kSeg, kRunCnt, kRunOff, kWpInv, kWTurns,
    kPrep, kFlag,
    kGroupInfo, kTwiddle, kPart, kNumBuf
};

std::mutex g_mutex;                  // one driver call at a time

// The HIP device of the calling thread: every cache below is per device
// (a process may drive several GPUs; device buffers and plans of one are
// not usable on another).
int current_device()
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    return dev;
}

Workspace& workspace()
{
    static std::map<int, Workspace> ws;
    return ws[current_device()];
}

sdp_fft::Plan2D* cached_plan(int n, bool dbl, size_t batch, size_t dist,
        sdp_Error* status)
{
    static std::map<std::tuple<int, int, bool, size_t, size_t>,
            sdp_fft::Plan2D*> cache;
    const auto key = std::make_tuple(current_device(), n, dbl, batch, dist);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    sdp_fft::Plan2D* p = sdp_fft::create_2d_batched(n, n, dbl, batch, dist,
            status);
    if (p) cache[key] = p;
    return p;
}

// The w-stack plane FFT (complex float, G a power of two in [1024, 16384]):
// the fused three-pass FFT (es_fft.hip) in place, output rows permuted,
// instead of rocFFT's four passes (rocFFT for f64 and other sizes).
const sdp_es::FftTwiddles* plane_fft_twiddles(int64_t G, bool dbl,
        sdp_Error* status)
{
    if (dbl || G > INT32_MAX || !sdp_es::fused_fft_supported((int)G))
        return nullptr;
    static std::map<std::pair<int, int64_t>, sdp_es::FftTwiddles> cache;
    const auto key = std::make_pair(current_device(), G);
    auto it = cache.find(key);
    if (it != cache.end()) return &it->second;
    sdp_es::FftTwiddles tw;
    if (sdp_es::fft_twiddles_create((int)G, &tw) != 0)
    {
        *status = SDP_ERR_RUNTIME;
        return nullptr;
    }
    return &(cache[key] = tw);
}

// Twiddles of the batched sub-grid FFT (es_fft_wstack.h subgrid_fft2d):
// complex-float sub-grids of S = 128 or 256 (rocFFT otherwise).
const sdp_es::FftTwiddles* subgrid_fft_twiddles(int S, bool dbl,
        sdp_Error* status)
{
    if (dbl || !sdp_es::subgrid_fft_supported(S)) return nullptr;
    static std::map<std::pair<int, int>, sdp_es::FftTwiddles> cache;
    const auto key = std::make_pair(current_device(), S);
    auto it = cache.find(key);
    if (it != cache.end()) return &it->second;
    sdp_es::FftTwiddles tw;
    if (sdp_es::fft_twiddles_create(S, &tw) != 0)
    {
        *status = SDP_ERR_RUNTIME;
        return nullptr;
    }
    return &(cache[key] = tw);
}

sdp_GridderWtowerUVW* cached_kernel(int image_size, int S, double theta,
        double w_step, double hu, double hv, int support, int os,
        int w_support, int wos, sdp_Error* status)
{
    static std::map<std::tuple<int, int, int, double, double, double,
            double, int, int, int, int>, sdp_GridderWtowerUVW*> cache;
    const auto key = std::make_tuple(current_device(), image_size, S, theta,
            w_step, hu, hv, support, os, w_support, wos);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    sdp_GridderWtowerUVW* k = sdp_gridder_wtower_uvw_create(image_size, S,
            theta, w_step, hu, hv, support, os, w_support, wos, status);
    if (!k) return nullptr;
    plan_ensure_correction(k, status);
    if (*status)
    {
        sdp_gridder_wtower_uvw_free(k);
        return nullptr;
    }
    cache[key] = k;
    return k;
}

// Correction parameters with the plan's cached per-pixel scale table, f32
// for float facets and f64 for double ones (built on first use; plans are
// cached for the process lifetime by cached_kernel).
CorrParams corr_params_tab(const sdp_GridderWtowerUVW* k, int w_offset,
        bool inverse, bool f32, sdp_Error* status)
{
    static std::map<std::pair<const void*, bool>, void*> tabs;
    CorrParams cp = corr_params(k, w_offset, inverse);
    const auto key = std::make_pair((const void*)k, f32);
    auto it = tabs.find(key);
    if (it == tabs.end())
    {
        const int64_t N = k->image_size;
        void* d = nullptr;
        if (hipMalloc(&d, N * N * (f32 ? sizeof(float) : sizeof(double))) !=
                hipSuccess)
        {
            (void)hipGetLastError();
            return cp;    // no room: evaluate per pixel
        }
        if (f32)
            k_scale_table<float><<<dim3(blocks_of(N), (unsigned)N), 256>>>(
                    cp, (float*)d);
        else
            k_scale_table<double><<<dim3(blocks_of(N), (unsigned)N), 256>>>(
                    cp, (double*)d);
        SDP_HIP_CHECK_LAUNCH(status);
        it = tabs.emplace(key, d).first;
    }
    if (f32) cp.scale_f32 = (const float*)it->second;
    else cp.scale_f64 = (const double*)it->second;
    return cp;
}

// One (w-stack plane, batch of sub-grids) unit of work.
struct Group
{
    int64_t iw;
    int64_t slots, slots_alloc;
    int64_t task_base;               // into the concatenated task list
    int64_t first_p, last_p;         // global w-layer range with items
    bool first_of_plane, last_of_plane;
};

struct Binned
{
    Geo g;
    std::vector<Group> groups;
    std::vector<int> tasks;          // concatenated slot -> task ids
    std::vector<int64_t> offsets;    // [groups][NP + 1] item offsets
    int4* items = nullptr;           // sorted
    const uint64_t* keys = nullptr;  // sorted keys
    int* d_tasks = nullptr;
    int64_t n_items = 0;
    int64_t t_cap = 0;
};

double now_s()
{
    return std::chrono::duration<double>(
            std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Bounds of all visibilities (sdp_gridder_uvw_bounds_all with all channels,
// .cpp:318-330), then the binning passes.
template<typename U>
bool bin_visibilities(const U* d_uvw, Geo& g, size_t budget_bytes,
        size_t per_slot_bytes, Binned* out, sdp_Error* status)
{
    Workspace& ws = workspace();
    const int64_t R = g.num_rows;
    int* d_s = (int*)ws.get(kBounds, 2 * R * sizeof(int), status);
    if (*status) return false;
    int* d_e = d_s + R;
    k_fill_int<<<blocks_of(2 * R), 256>>>(d_s, R, 0, (int)g.num_chan);
    SDP_HIP_CHECK_LAUNCH(status);
    double lo[3], hi[3];
    uvw_bounds_dev<U>(d_uvw, R, g.f0, g.df, d_s, d_e, lo, hi, status);
    if (*status) return false;
    if (!(lo[0] <= hi[0])) return false;          // no visibilities
    const double eta = 1e-5;
    g.min_iu = (int64_t)floor(lo[0] / g.eff_dist + 0.5 - eta);
    g.max_iu = (int64_t)floor(hi[0] / g.eff_dist + 0.5 + eta);
    g.min_iv = (int64_t)floor(lo[1] / g.eff_dist + 0.5 - eta);
    g.max_iv = (int64_t)floor(hi[1] / g.eff_dist + 0.5 + eta);
    g.min_iw = (int64_t)floor(lo[2] / g.ws_dist + 0.5 - eta);
    g.max_iw = (int64_t)floor(hi[2] / g.ws_dist + 0.5 + eta);
    g.nu = g.max_iu - g.min_iu + 1;
    g.nv = g.max_iv - g.min_iv + 1;
    g.niw = g.max_iw - g.min_iw + 1;
    g.ntask = g.nu * g.nv;
    g.P0 = (int64_t)floor(fmin(lo[2], hi[2]) / g.w_step) - 2;
    g.NP = (int64_t)floor(hi[2] / g.w_step) + 4 - g.P0;
    if (g.nu * g.nv * g.niw > (int64_t)1 << 31)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Too many sub-grids (%lld x %lld x %lld w-planes)",
                (long long)g.nu, (long long)g.nv, (long long)g.niw);
        return false;
    }

    // Count pass.
    int64_t* d_count = (int64_t*)ws.get(kRowCount, (R + 1) * sizeof(int64_t),
            status);
    unsigned char* d_occ = (unsigned char*)ws.get(kOccupied,
            g.niw * g.ntask, status);
    if (*status) return false;
    SDP_HIP_CHECK(hipMemsetAsync(d_occ, 0, g.niw * g.ntask, 0), status);
    BinOut bo = {};
    bo.row_count = d_count;
    bo.occupied = d_occ;
    k_bin<U, false><<<blocks_of(R), 256>>>(d_uvw, g, bo);
    SDP_HIP_CHECK_LAUNCH(status);
    // Row offsets (exclusive scan of the counts).
    int64_t* d_off = (int64_t*)ws.get(kRowOffset, (R + 1) * sizeof(int64_t),
            status);
    size_t temp_bytes = 0;
    SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, temp_bytes,
            d_count, d_off, (int)(R + 1)), status);
    void* d_temp = ws.get(kTemp, temp_bytes, status);
    if (*status) return false;
    SDP_HIP_CHECK(hipMemsetAsync(d_count + R, 0, sizeof(int64_t), 0),
            status);
    SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(d_temp, temp_bytes,
            d_count, d_off, (int)(R + 1)), status);
    int64_t n_items = 0;
    SDP_HIP_CHECK(hipMemcpy(&n_items, d_off + R, sizeof(int64_t),
            hipMemcpyDeviceToHost), status);
    std::vector<unsigned char> occ(g.niw * g.ntask);
    SDP_HIP_CHECK(hipMemcpy(occ.data(), d_occ, occ.size(),
            hipMemcpyDeviceToHost), status);
    if (*status) return false;
    if (n_items > 0x7FFFFFFF)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Too many visibility runs (%lld)", (long long)n_items);
        return false;
    }

    // Groups: the sub-grids of each w-stack plane, in task order, in
    // batches within the memory budget.
    const int64_t max_slots = std::max<int64_t>(1,
            (int64_t)(budget_bytes / per_slot_bytes));
    std::vector<Slot> slot_map(g.niw * g.ntask, Slot{-1, -1});
    out->groups.clear();
    out->tasks.clear();
    for (int64_t iw_rel = 0; iw_rel < g.niw; ++iw_rel)
    {
        std::vector<int> list;
        for (int64_t t = 0; t < g.ntask; ++t)
            if (occ[iw_rel * g.ntask + t]) list.push_back((int)t);
        for (size_t b = 0; b < list.size(); b += max_slots)
        {
            Group gr;
            gr.iw = g.min_iw + iw_rel;
            gr.slots = std::min<int64_t>(max_slots, list.size() - b);
            gr.slots_alloc = (gr.slots + 63) / 64 * 64;
            gr.task_base = (int64_t)out->tasks.size();
            gr.first_of_plane = (b == 0);
            gr.last_of_plane = (b + gr.slots == list.size());
            gr.first_p = gr.last_p = 0;
            for (int64_t s = 0; s < gr.slots; ++s)
            {
                const int t = list[b + s];
                out->tasks.push_back(t);
                slot_map[iw_rel * g.ntask + t] =
                        Slot{(int)out->groups.size(), (int)s};
            }
            out->groups.push_back(gr);
        }
    }
    const int64_t ng = (int64_t)out->groups.size();
    out->t_cap = 64;
    for (const Group& gr : out->groups)
        out->t_cap = std::max(out->t_cap, gr.slots_alloc);
    out->n_items = n_items;
    out->g = g;
    if (ng == 0 || n_items == 0) return true;

    // Emit pass.
    Slot* d_map = (Slot*)ws.get(kSlotMap, slot_map.size() * sizeof(Slot),
            status);
    uint64_t* d_keys = (uint64_t*)ws.get(kKeys, n_items * 8, status);
    uint64_t* d_keys2 = (uint64_t*)ws.get(kKeysAlt, n_items * 8, status);
    uint32_t* d_idx = (uint32_t*)ws.get(kIdx, n_items * 4, status);
    uint32_t* d_idx2 = (uint32_t*)ws.get(kIdxAlt, n_items * 4, status);
    int4* d_raw = (int4*)ws.get(kItemsRaw, n_items * sizeof(int4), status);
    int4* d_items = (int4*)ws.get(kItems, n_items * sizeof(int4), status);
    unsigned int* d_hist = (unsigned int*)ws.get(kHist,
            ng * g.NP * sizeof(unsigned int), status);
    int* d_tasks = (int*)ws.get(kTasks, out->tasks.size() * sizeof(int),
            status);
    if (*status) return false;
    SDP_HIP_CHECK(hipMemcpy(d_map, slot_map.data(),
            slot_map.size() * sizeof(Slot), hipMemcpyHostToDevice), status);
    SDP_HIP_CHECK(hipMemcpy(d_tasks, out->tasks.data(),
            out->tasks.size() * sizeof(int), hipMemcpyHostToDevice), status);
    SDP_HIP_CHECK(hipMemsetAsync(d_hist, 0, ng * g.NP * sizeof(unsigned int),
            0), status);
    bo = {};
    bo.row_offset = d_off;
    bo.slot_map = d_map;
    bo.keys = d_keys;
    bo.idx = d_idx;
    bo.items = d_raw;
    bo.hist = d_hist;
    bo.t_cap = out->t_cap;
    k_bin<U, true><<<blocks_of(R), 256>>>(d_uvw, g, bo);
    SDP_HIP_CHECK_LAUNCH(status);
    // Sort by (group, w-layer, slot).
    const uint64_t max_key = ((uint64_t)ng * g.NP) * out->t_cap;
    int end_bit = 1;
    while (end_bit < 64 && (max_key >> end_bit)) ++end_bit;
    hipcub::DoubleBuffer<uint64_t> kb(d_keys, d_keys2);
    hipcub::DoubleBuffer<uint32_t> vb(d_idx, d_idx2);
    temp_bytes = 0;
    SDP_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes,
            kb, vb, (int)n_items, 0, end_bit), status);
    d_temp = ws.get(kTemp, temp_bytes, status);
    if (*status) return false;
    SDP_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(d_temp, temp_bytes,
            kb, vb, (int)n_items, 0, end_bit), status);
    k_gather_items<<<blocks_of(n_items), 256>>>(vb.Current(), d_raw, d_items,
            n_items);
    out->keys = kb.Current();
    SDP_HIP_CHECK_LAUNCH(status);
    // Item offsets per (group, w-layer).
    std::vector<unsigned int> hist(ng * g.NP);
    SDP_HIP_CHECK(hipMemcpy(hist.data(), d_hist, hist.size() * 4,
            hipMemcpyDeviceToHost), status);
    if (*status) return false;
    out->offsets.assign(ng * (g.NP + 1), 0);
    int64_t run = 0;
    for (int64_t gi = 0; gi < ng; ++gi)
    {
        Group& gr = out->groups[gi];
        gr.first_p = -1;
        for (int64_t p = 0; p < g.NP; ++p)
        {
            out->offsets[gi * (g.NP + 1) + p] = run;
            const unsigned int c = hist[gi * g.NP + p];
            if (c)
            {
                if (gr.first_p < 0) gr.first_p = p;
                gr.last_p = p;
            }
            run += c;
        }
        out->offsets[gi * (g.NP + 1) + g.NP] = run;
    }
    out->items = d_items;
    out->d_tasks = d_tasks;
    return true;
}

TowerParams tower_params(const sdp_GridderWtowerUVW* k, const Geo& g,
        const Group& gr, const Binned& b)
{
    TowerParams p;
    p.S = g.S;
    p.support = k->support;
    p.w_support = k->w_support;
    p.os = k->oversampling;
    p.wos = k->w_oversampling;
    p.theta = g.theta;
    p.w_step = g.w_step;
    p.f0 = g.f0;
    p.df = g.df;
    p.num_chan = g.num_chan;
    p.off_w = (int)(gr.iw * g.H);
    p.w_plane = 0;
    p.ring = 0;
    p.layer = (int64_t)g.S * g.S;
    p.layer_stride = p.layer * gr.slots_alloc;
    p.task = b.d_tasks + gr.task_base;
    p.nv = g.nv;
    p.min_iu = g.min_iu;
    p.min_iv = g.min_iv;
    p.eff = g.eff;
    return p;
}


struct DftData
{
    int4* vrec = nullptr;
    int* seg_start = nullptr;
    int* seg_end = nullptr;
    Cx<double>* wp_inv = nullptr;
    double* w_turns = nullptr;
    float* prep = nullptr;
    int prep_stride = 0;
    float2* tw = nullptr;
    int64_t n_vis = 0;
};

// Channel records in (group, slot, layer) order, per-slot segments, 1 / D;
// false (fall back to the layer-by-layer path) if a tower is deeper than
// kDftLayers or a visibility's taps leave its sub-grid.
template<typename U>
bool prepare_dft(const sdp_GridderWtowerUVW* k, const U* d_uvw,
        const Cx<float>* d_vis_in, const Binned& b, DftData* dd,
        sdp_Error* status)
{
    Workspace& ws = workspace();
    const Geo& g = b.g;
    const int64_t ng = (int64_t)b.groups.size();
    for (const Group& gr : b.groups)
        if (gr.first_p >= 0 && gr.last_p - gr.first_p + 1 > kDftLayers)
            return false;
    const int64_t n = b.n_items;
    int64_t* d_cnt = (int64_t*)ws.get(kRunCnt, (n + 1) * sizeof(int64_t),
            status);
    int64_t* d_off = (int64_t*)ws.get(kRunOff, (n + 1) * sizeof(int64_t),
            status);
    if (*status) return false;
    k_run_channels<<<blocks_of(n), 256>>>(b.items, n, d_cnt);
    SDP_HIP_CHECK(hipMemsetAsync(d_cnt + n, 0, sizeof(int64_t), 0), status);
    size_t temp_bytes = 0;
    SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, temp_bytes,
            d_cnt, d_off, (int)(n + 1)), status);
    void* d_temp = ws.get(kTemp, temp_bytes, status);
    if (*status) return false;
    SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(d_temp, temp_bytes,
            d_cnt, d_off, (int)(n + 1)), status);
    int64_t n_vis = 0;
    SDP_HIP_CHECK(hipMemcpy(&n_vis, d_off + n, sizeof(int64_t),
            hipMemcpyDeviceToHost), status);
    if (*status || n_vis > 0x7FFFFFFF) return false;
    dd->vrec = (int4*)ws.get(kVrec, std::max<int64_t>(n_vis, 1) *
            sizeof(int4), status);
    const int64_t nseg = ng * b.t_cap;
    dd->seg_start = (int*)ws.get(kSeg, 2 * nseg * sizeof(int), status);
    dd->wp_inv = (Cx<double>*)ws.get(kWpInv,
            (size_t)g.S * g.S * sizeof(Cx<double>), status);
    dd->w_turns = (double*)ws.get(kWTurns, (size_t)g.S * g.S * sizeof(double),
            status);
    dd->prep_stride = prep_stride(g.support);
    dd->prep = (float*)ws.get(kPrep, (size_t)std::max<int64_t>(n_vis, 1) *
            dd->prep_stride * sizeof(float), status);
    int* d_flag = (int*)ws.get(kFlag, sizeof(int), status);
    dd->tw = (float2*)ws.get(kTwiddle, g.S * sizeof(float2), status);
    int* d_ginfo = (int*)ws.get(kGroupInfo, 2 * ng * sizeof(int), status);
    if (*status) return false;
    dd->seg_end = dd->seg_start + nseg;
    dd->n_vis = n_vis;
    k_expand_runs<<<blocks_of(n), 256>>>(b.items, b.keys, d_off, n, g.NP,
            dd->vrec);
    SDP_HIP_CHECK(hipMemsetAsync(dd->seg_start, 0, 2 * nseg * sizeof(int),
            0), status);
    if (n_vis > 0)
        k_segments<<<blocks_of(n_vis), 256>>>(dd->vrec, n_vis,
                dd->seg_start, dd->seg_end);
    k_twiddles<<<blocks_of(g.S), 256>>>(dd->tw, g.S);
    k_pattern_inv<<<blocks_of((int64_t)g.S * g.S), 256>>>(
            (const Cx<double>*)k->d_w_pattern, dd->wp_inv,
            (int64_t)g.S * g.S);
    k_pattern_turns<<<blocks_of((int64_t)g.S * g.S), 256>>>(dd->w_turns,
            g.S, k->theta, k->shear_u, k->shear_v, k->w_step);
    std::vector<int> ginfo(2 * ng);
    for (int64_t gi = 0; gi < ng; ++gi)
    {
        ginfo[gi] = (int)(b.groups[gi].iw * g.H);
        ginfo[ng + gi] = (int)b.groups[gi].task_base;
    }
    SDP_HIP_CHECK(hipMemcpy(d_ginfo, ginfo.data(), ginfo.size() * sizeof(int),
            hipMemcpyHostToDevice), status);
    SDP_HIP_CHECK(hipMemsetAsync(d_flag, 0, sizeof(int), 0), status);
    if (n_vis > 0)
    {
        const TowerParams base = tower_params(k, g, b.groups[0], b);
        k_dft_prep<U><<<blocks_of(n_vis), 256>>>(dd->vrec, n_vis, d_uvw,
                d_vis_in, base, b.d_tasks, d_ginfo, d_ginfo + ng, b.t_cap,
                g.P0, k->d_uv_kernel, k->d_w_kernel, dd->prep, d_flag);
    }
    SDP_HIP_CHECK_LAUNCH(status);
    int flag = 0;
    SDP_HIP_CHECK(hipMemcpy(&flag, d_flag, sizeof(int),
            hipMemcpyDeviceToHost), status);
    return !*status && flag == 0;
}

struct Timing
{
    double bin = 0, towers = 0, image = 0;
    int64_t layers = 0;
};

// Device timing of the fused tower kernels (k_tower_dft / k_tower_idft),
// switched on by sdp_grid_wstack_wtower_enable_timing: one HIP event pair
// per launch on the launch stream, read back at the end of the call, plus
// the work counts the roofline needs (visibilities, sub-grid w-layers).
struct TowerTiming
{
    bool on = false;
    std::vector<hipEvent_t> ev;     // start/stop pairs, reused across calls
    size_t used = 0;
    double ms = 0;
    int64_t launches = 0, vis = 0, layers = 0;
    int S = 0, kind = 0;            // kind: 0 gridding, 1 degridding

    void start()
    {
        if (!on) return;
        while (ev.size() < used + 2)
        {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) { on = false; return; }
            ev.push_back(e);
        }
        (void)hipEventRecord(ev[used], 0);
    }
    void stop()
    {
        if (!on || ev.size() < used + 2) return;
        (void)hipEventRecord(ev[used + 1], 0);
        used += 2;
        ++launches;
    }
    void collect()
    {
        for (size_t i = 0; i + 1 < used; i += 2)
        {
            float t = 0.f;
            if (hipEventSynchronize(ev[i + 1]) == hipSuccess &&
                    hipEventElapsedTime(&t, ev[i], ev[i + 1]) == hipSuccess)
                ms += t;
        }
        used = 0;
    }
};

TowerTiming& tower_timing()
{
    static TowerTiming t;
    return t;
}


// Grid all visibilities of the selected w-stack planes.
template<typename T, typename U>
void grid_all_impl(sdp_GridderWtowerUVW* k, Geo g, const Cx<T>* d_vis,
        const U* d_uvw, AnyView image, int64_t G, int verbosity,
        sdp_Error* status)
{
    Workspace& ws = workspace();
    Timing tm;
    double t0 = now_s();
    const int64_t layer = (int64_t)g.S * g.S;
    const size_t per_slot = layer * (size_t)(g.w_support * sizeof(Cx<T>) +
            sizeof(Cx<double>));
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    const size_t budget = std::max<size_t>(per_slot * 64, free_b / 3);
    Binned b;
    g.fused = (sizeof(T) == 4 && g.S % kDftTile == 0 &&
            g.S <= kDftMaxS && g.w_support <= 16 && g.support <= 16) ? 1 : 0;
    bool any = bin_visibilities<U>(d_uvw, g, budget, per_slot, &b, status);
    if (*status) return;
    DftData dd;
    if (b.g.fused && any && !b.groups.empty() && b.n_items > 0 &&
            !prepare_dft<U>(k, d_uvw, sizeof(T) == 4 ?
                    (const Cx<float>*)(const void*)d_vis : nullptr, b, &dd,
                    status))
    {
        if (*status) return;
        g.fused = 0;    // layer-by-layer path: re-bin in (layer, slot) order
        any = bin_visibilities<U>(d_uvw, g, budget, per_slot, &b, status);
        if (*status) return;
    }
    if (verbosity > 0)
    {
        (void)hipDeviceSynchronize();
        tm.bin = now_s() - t0;
    }
    g = b.g;
    if (!any || b.groups.empty()) return;
    Cx<T>* d_stack = (Cx<T>*)ws.get(kStack,
            b.t_cap * layer * g.w_support * sizeof(Cx<T>), status);
    Cx<double>* d_wimg = (Cx<double>*)ws.get(kWimg,
            b.t_cap * layer * sizeof(Cx<double>), status);
    Cx<T>* d_grid = (Cx<T>*)ws.get(kGrid, G * G * sizeof(Cx<T>), status);
    // Task -> slot maps of all groups, uploaded once: a per-group
    // hipMemcpyAsync from one reused pageable host vector raced with its
    // refill for the next group while earlier kernels were still queued.
    const int64_t ngr = (int64_t)b.groups.size();
    int* d_slot_of = (int*)ws.get(kSlotOf, ngr * g.ntask * sizeof(int),
            status);
    sdp_fft::Plan2D* big = cached_plan((int)G, sizeof(T) == 8, 1, G * G,
            status);
    if (*status) return;
    const Cx<double>* wp = (const Cx<double>*)k->d_w_pattern;
    const int ws_n = g.w_support;
    const T factor = (T)((double)k->image_size / g.S *
            ((double)k->image_size / g.S));
    if (!*status)
    {
        std::vector<int> slot_of(ngr * g.ntask, -1);
        for (int64_t gi = 0; gi < ngr; ++gi)
            for (int64_t sl = 0; sl < b.groups[gi].slots; ++sl)
                slot_of[gi * g.ntask + b.tasks[b.groups[gi].task_base + sl]] =
                        (int)sl;
        SDP_HIP_CHECK(hipMemcpy(d_slot_of, slot_of.data(),
                slot_of.size() * sizeof(int), hipMemcpyHostToDevice), status);
    }
    for (size_t gi = 0; gi < b.groups.size() && !*status; ++gi)
    {
        const Group& gr = b.groups[gi];
        const double tg = now_s();
        if (verbosity > 1)
            SDP_LOG_INFO("group %zu: w-stack plane %lld, %lld sub-grids, "
                    "w-layers %lld..%lld (relative), items %lld..%lld", gi,
                    (long long)gr.iw, (long long)gr.slots,
                    (long long)(gr.first_p + g.P0 - (int)(gr.iw * g.H)),
                    (long long)(gr.last_p + g.P0 - (int)(gr.iw * g.H)),
                    (long long)b.offsets[gi * (g.NP + 1)],
                    (long long)b.offsets[gi * (g.NP + 1) + g.NP]);
        sdp_fft::Plan2D* sp = cached_plan(g.S, sizeof(T) == 8,
                gr.slots_alloc, layer, status);
        if (*status) break;
        TowerParams p = tower_params(k, g, gr, b);
        const int64_t n_el = gr.slots * layer;
        const int64_t ls = p.layer_stride;
        const bool empty = gr.first_p < 0;   // no visibility survived
        if (g.fused && !empty)
        {
            if constexpr (sizeof(T) == 4)
            {
                DftParams dp;
                dp.tp = p;
                dp.vrec = dd.vrec;
                dp.seg_start = dd.seg_start;
                dp.seg_end = dd.seg_end;
                dp.gslot_base = (int64_t)gi * b.t_cap;
                dp.P0 = g.P0;
                dp.out = (Cx<float>*)d_stack;
                dp.wp = wp;
                dp.wp_inv = dd.wp_inv;
                dp.w_turns = dd.w_turns;
                dp.prep = dd.prep;
                dp.prep_stride = dd.prep_stride;
                dp.uv_kernel = k->d_uv_kernel;
                dp.w_kernel = k->d_w_kernel;
                dp.tw = dd.tw;
                // Two 16 x 16 blocks per wave where the sub-grid allows.
                const bool two = g.S % (2 * kDftTile) == 0;
                const int tiles = (g.S / kDftTile) *
                        (g.S / (two ? 2 * kDftTile : kDftTile));
                tower_timing().start();
                if (two)
                    k_tower_dft<U, 2><<<dim3(tiles, (unsigned)gr.slots),
                            256, g.S * sizeof(float2)>>>(dp, d_uvw,
                            (const Cx<float>*)d_vis);
                else
                    k_tower_dft<U, 1><<<dim3(tiles, (unsigned)gr.slots),
                            256, g.S * sizeof(float2)>>>(dp, d_uvw,
                            (const Cx<float>*)d_vis);
                SDP_HIP_CHECK_LAUNCH(status);
                tower_timing().stop();
                const sdp_es::FftTwiddles* stw = subgrid_fft_twiddles(g.S,
                        false, status);
                if (stw)
                {
                    const int e = sdp_es::subgrid_fft2d((float*)d_stack, g.S,
                            gr.slots, true, *stw, nullptr, 0);
                    if (e) *status = (sdp_Error)e;
                }
                else
                {
                    sdp_fft::exec_2d(sp, d_stack, true, 0, status);
                }
            }
            tm.layers += (gr.last_p - gr.first_p + ws_n) * gr.slots;
        }
        else if (g.fused)
        {
            SDP_HIP_CHECK(hipMemsetAsync(d_stack, 0,
                    gr.slots_alloc * layer * sizeof(Cx<T>), 0), status);
        }
        if (!g.fused)
        {
            SDP_HIP_CHECK(hipMemsetAsync(d_stack, 0,
                    gr.slots_alloc * layer * ws_n * sizeof(Cx<T>), 0), status);
            SDP_HIP_CHECK(hipMemsetAsync(d_wimg, 0, n_el * sizeof(Cx<double>),
                    0), status);
            const int64_t first = empty ? 0 : gr.first_p + g.P0 - p.off_w;
            const int64_t last = empty ? -1 : gr.last_p + g.P0 - p.off_w;
            int ring = 0;
            for (int64_t w_plane = first; w_plane <= last && !*status; ++w_plane)
            {
                if (w_plane != first)
                {
                    sdp_fft::exec_2d(sp, d_stack + ring * ls, false, 0, status);
                    k_grid_step<T><<<blocks_of(n_el), 256>>>(d_wimg,
                            d_stack + ring * ls, wp, layer, g.S, n_el, 1);
                    ring = (ring + 1) % ws_n;
                }
                const int64_t prel = w_plane + p.off_w - g.P0;
                const int64_t i0 = b.offsets[gi * (g.NP + 1) + prel];
                const int64_t i1 = b.offsets[gi * (g.NP + 1) + prel + 1];
                if (i1 > i0)
                {
                    p.w_plane = (int)w_plane;
                    p.ring = ring;
                    k_tower_grid<T, U><<<blocks_of(i1 - i0, kWaves),
                            64 * kWaves>>>(p, b.items + i0, i1 - i0, d_uvw,
                            d_stack, k->d_uv_kernel, k->d_w_kernel, d_vis);
                }
                SDP_HIP_CHECK_LAUNCH(status);
            }
            for (int i = 0; i < ws_n && !*status && !empty; ++i)
            {
                const int l = (ring + i) % ws_n;
                sdp_fft::exec_2d(sp, d_stack + l * ls, false, 0, status);
                k_grid_step<T><<<blocks_of(n_el), 256>>>(d_wimg, d_stack + l * ls,
                        wp, layer, g.S, n_el, 0);
            }
            tm.layers += (last - first + 1) * gr.slots;
            if (!empty)
            {
                k_grid_final<T><<<blocks_of(n_el), 256>>>(d_wimg, d_stack, wp,
                        layer, g.S, (int)(last + ws_n / 2 - 1), n_el);
                sdp_fft::exec_2d(sp, d_stack, true, 0, status);
            }
        }
        // Sub-grids into the grid.
        // Sub-grids covering a cell per axis: ceil(S / eff) per periodic
        // image of the cell (x - G, x, x + G) that falls inside the axis'
        // sub-grid span L = (n - 1) eff + S; at most floor(L / G) + 1 of
        // the three do (a uvw extent wider than the grid wraps onto it).
        auto axis_cand = [&](int64_t n_idx) {
            const int64_t L = (n_idx - 1) * g.eff + g.S;
            const int64_t wraps = std::min<int64_t>(3, L / G + 1);
            return (int)(((g.S + g.eff - 1) / g.eff) * wraps);
        };
        const int ncand = std::max(axis_cand(g.nu), axis_cand(g.nv));
        // No-wrap gather when every sub-grid of both axes lies inside the
        // grid (k_gather_grid_nw).
        auto inside = [&](int64_t min_i, int64_t n_idx) {
            const int64_t first = G / 2 - g.S / 2 + min_i * g.eff;
            const int64_t last = first + (n_idx - 1) * g.eff + g.S - 1;
            return first >= 0 && last <= G - 1;
        };
        const int nc_nw = (int)((g.S + g.eff - 1) / g.eff);
        const bool nowrap = inside(g.min_iu, g.nu) && inside(g.min_iv, g.nv)
                && nc_nw <= 3 && G < (1 << 30);
        // The plane's last group with the fused f32 plane FFT: the image
        // update runs inside the FFT's last column pass (es_fft_wstack.h).
        // (A gather fused into the row pass measured 10.3 ms per plane at
        // config 4 against 2.0 + 0.9 ms for the gather and the row pass:
        // one 512-thread workgroup per CU cannot hide the dependent
        // slot-table and sub-grid loads; the gather stays its own pass.)
        const sdp_es::FftTwiddles* tw_plane = (gr.last_of_plane &&
                sizeof(T) == 4) ? plane_fft_twiddles(G, false, status) :
                nullptr;
        if (*status) break;
        const dim3 gnw(blocks_of(G), (unsigned)((G + kGatherRows - 1) /
                kGatherRows));
        if (nowrap && nc_nw <= 2)
            k_gather_grid_nw<T, 2><<<gnw, 256>>>(d_grid, (int)G, d_stack,
                    g.S, d_slot_of + gi * g.ntask, (int)g.nu, (int)g.nv,
                    (int)g.min_iu, (int)g.min_iv, g.eff, factor,
                    gr.first_of_plane ? 0 : 1);
        else if (nowrap)
            k_gather_grid_nw<T, 3><<<gnw, 256>>>(d_grid, (int)G, d_stack,
                    g.S, d_slot_of + gi * g.ntask, (int)g.nu, (int)g.nv,
                    (int)g.min_iu, (int)g.min_iv, g.eff, factor,
                    gr.first_of_plane ? 0 : 1);
        else if (ncand <= 3)
            k_gather_grid<T, 3><<<dim3(blocks_of(G), (unsigned)G), 256>>>(
                    d_grid, G, d_stack, g.S, d_slot_of + gi * g.ntask, g.nu,
                    g.nv, g.min_iu, g.min_iv, g.eff, factor,
                    gr.first_of_plane ? 0 : 1);
        else if (ncand <= 8)
            k_gather_grid<T, 8><<<dim3(blocks_of(G), (unsigned)G), 256>>>(
                    d_grid, G, d_stack, g.S, d_slot_of + gi * g.ntask, g.nu,
                    g.nv, g.min_iu, g.min_iv, g.eff, factor,
                    gr.first_of_plane ? 0 : 1);
        else
        {
            *status = SDP_ERR_INVALID_ARGUMENT;
            SDP_LOG_ERROR("subgrid_frac too small: %d sub-grids overlap",
                    ncand - 1);
            break;
        }
        SDP_HIP_CHECK_LAUNCH(status);
        if (verbosity > 0)
        {
            (void)hipDeviceSynchronize();
            tm.towers += now_s() - tg;
        }
        if (gr.last_of_plane && tw_plane)
        {
            const double ti = now_s();
            const CorrParams cp = corr_params_tab(k, (int)(gr.iw * g.H), true,
                    true, status);
            if (*status) break;
            const int e = sdp_es::fft2d_wstack_grid_image((float*)d_grid,
                    (int)G, *tw_plane, image,
                    (float)(1.0 / ((double)G * G)), cp, 0);
            if (e) { *status = (sdp_Error)e; break; }
            if (verbosity > 0)
            {
                (void)hipDeviceSynchronize();
                tm.image += now_s() - ti;
            }
        }
        else if (gr.last_of_plane)
        {
            const double ti = now_s();
            const sdp_es::FftTwiddles* tw = plane_fft_twiddles(G,
                    sizeof(T) == 8, status);
            int perm_n2 = 0;
            if (tw)
            {
                const int e = sdp_es::fft2d_inplace_permuted((float*)d_grid,
                        (int)G, false, *tw, 0);
                if (e) *status = (sdp_Error)e;
                perm_n2 = sdp_es::fft_perm_n2((int)G);
            }
            else
            {
                sdp_fft::exec_2d(big, d_grid, false, 0, status);
            }
            const CorrParams cp = corr_params_tab(k, (int)(gr.iw * g.H), true,
                    sizeof(T) == 4, status);
            k_image_update<T><<<dim3(blocks_of(G),
                    (unsigned)((G + kImgRows - 1) / kImgRows)), 256>>>(
                    d_grid, G, image, (T)(1.0 / ((double)G * G)), cp,
                    perm_n2);
            SDP_HIP_CHECK_LAUNCH(status);
            if (verbosity > 0)
            {
                (void)hipDeviceSynchronize();
                tm.image += now_s() - ti;
            }
        }
    }
    if (tower_timing().on && g.fused)
    {
        TowerTiming& tt = tower_timing();
        tt.collect();
        tt.vis += dd.n_vis;
        tt.layers += tm.layers;
        tt.S = g.S;
        tt.kind = 0;
    }
    if (verbosity > 0 && !*status)
    {
        SDP_LOG_INFO("w-stacking with w-towers (gridding): %lld w-stack "
                "planes, %lld sub-grids x %lld, %zu sub-grid groups, %lld "
                "visibility runs, %lld sub-grid w-layers",
                (long long)g.niw, (long long)g.nu, (long long)g.nv,
                b.groups.size(), (long long)b.n_items, (long long)tm.layers);
        SDP_LOG_INFO("| binning %.3f s | towers %.3f s | image side %.3f s"
                " | %s", tm.bin, tm.towers, tm.image, g.fused ?
                "fused towers (k_tower_dft)" : "layer-by-layer towers");
    }
}

// Degrid all visibilities of the selected w-stack planes.
template<typename T, typename U>
void degrid_all_impl(sdp_GridderWtowerUVW* k, Geo g, AnyView image,
        int64_t G, const U* d_uvw, Cx<T>* d_vis, int verbosity,
        sdp_Error* status)
{
    Workspace& ws = workspace();
    Timing tm;
    double t0 = now_s();
    const int64_t layer = (int64_t)g.S * g.S;
    const size_t per_slot = layer * (size_t)((g.w_support + 1) *
            sizeof(Cx<T>));
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    const size_t budget = std::max<size_t>(per_slot * 64, free_b / 3);
    Binned b;
    g.fused = (sizeof(T) == 4 && g.S % kDftTile == 0 &&
            g.S <= kDftMaxS && g.w_support <= 16 && g.support <= 16) ? 1 : 0;
    bool any = bin_visibilities<U>(d_uvw, g, budget, per_slot, &b, status);
    if (*status) return;
    DftData dd;
    // Two 16 x 16 blocks per wave (32 x 64 tiles) where the sub-grid allows.
    const bool two = g.S % (2 * kDftTile) == 0;
    const int ntiles = (g.S / kDftTile) *
            (g.S / (two ? 2 * kDftTile : kDftTile));
    float2* d_part = nullptr;
    if (b.g.fused && any && !b.groups.empty() && b.n_items > 0)
    {
        bool ok = prepare_dft<U>(k, d_uvw, nullptr, b, &dd, status);
        if (*status) return;
        const size_t part_bytes = (size_t)std::max<int64_t>(dd.n_vis, 1) *
                ntiles * sizeof(float2);
        if (ok && part_bytes <= free_b / 3)
        {
            d_part = (float2*)ws.get(kPart, part_bytes, status);
            SDP_HIP_CHECK(hipMemsetAsync(d_part, 0, part_bytes, 0), status);
            if (*status) return;
        }
        else
        {
            g.fused = 0;   // layer-by-layer path: re-bin in (layer, slot) order
            any = bin_visibilities<U>(d_uvw, g, budget, per_slot, &b,
                    status);
            if (*status) return;
        }
    }
    if (verbosity > 0)
    {
        (void)hipDeviceSynchronize();
        tm.bin = now_s() - t0;
    }
    g = b.g;
    if (!any || b.groups.empty()) return;
    Cx<T>* d_stack = (Cx<T>*)ws.get(kStack,
            b.t_cap * layer * g.w_support * sizeof(Cx<T>), status);
    Cx<T>* d_wimg = (Cx<T>*)ws.get(kWimg, b.t_cap * layer * sizeof(Cx<T>),
            status);
    Cx<T>* d_grid = (Cx<T>*)ws.get(kGrid, G * G * sizeof(Cx<T>), status);
    sdp_fft::Plan2D* big = cached_plan((int)G, sizeof(T) == 8, 1, G * G,
            status);
    if (*status) return;
    const sdp_es::FftTwiddles* tw = plane_fft_twiddles(G, sizeof(T) == 8,
            status);
    if (*status) return;
    const int perm_n2 = tw ? sdp_es::fft_perm_n2((int)G) : 0;
    const Cx<double>* wp = (const Cx<double>*)k->d_w_pattern;
    const int ws_n = g.w_support;
    const T norm = (T)(1.0 / ((double)g.S * g.S));
    for (size_t gi = 0; gi < b.groups.size() && !*status; ++gi)
    {
        const Group& gr = b.groups[gi];
        if (gr.first_of_plane)
        {
            const double ti = now_s();
            const CorrParams cp = corr_params_tab(k, (int)(gr.iw * g.H),
                    false, sizeof(T) == 4, status);
            // (The image prologue fused into the plane FFT's row pass,
            // es_fft_wstack.h, measured 3.5 ms per plane at config 4
            // against 1.8 + 0.9 ms for the two passes: the per-element
            // double-precision correction starves the row pass's one
            // workgroup per CU.)
            if (tw)
            {
                // Complex float: the prologue is read by the plane FFT's
                // first (column) pass (es_fft_wstack.h).
                const int e = sdp_es::fft2d_wstack_image_to_grid(
                        (float*)d_grid, (int)G, *tw, image, cp, 0);
                if (e) *status = (sdp_Error)e;
            }
            else
            {
                k_image_to_grid<T><<<dim3(blocks_of(G),
                        (unsigned)((G + kImgRows - 1) / kImgRows)), 256>>>(
                        image, G, d_grid, cp);
                SDP_HIP_CHECK_LAUNCH(status);
                sdp_fft::exec_2d(big, d_grid, true, 0, status);
            }
            if (verbosity > 0)
            {
                (void)hipDeviceSynchronize();
                tm.image += now_s() - ti;
            }
        }
        const double tg = now_s();
        if (verbosity > 1)
            SDP_LOG_INFO("group %zu: w-stack plane %lld, %lld sub-grids, "
                    "w-layers %lld..%lld (relative), items %lld..%lld", gi,
                    (long long)gr.iw, (long long)gr.slots,
                    (long long)(gr.first_p + g.P0 - (int)(gr.iw * g.H)),
                    (long long)(gr.last_p + g.P0 - (int)(gr.iw * g.H)),
                    (long long)b.offsets[gi * (g.NP + 1)],
                    (long long)b.offsets[gi * (g.NP + 1) + g.NP]);
        if (gr.first_p < 0) continue;        // no visibility survived
        sdp_fft::Plan2D* sp = cached_plan(g.S, sizeof(T) == 8,
                gr.slots_alloc, layer, status);
        if (*status) break;
        TowerParams p = tower_params(k, g, gr, b);
        const int64_t n_el = gr.slots * layer;
        const int64_t ls = p.layer_stride;
        // Fused f32 towers with S = 128 / 256 (even G): the cut-out is read
        // by the first pass of the batched sub-grid FFT (es_fft_wstack.h);
        // otherwise k_cut_out + rocFFT.
        const sdp_es::FftTwiddles* stw = (g.fused && G % 2 == 0 &&
                G < (1 << 30) && sizeof(T) == 4) ?
                subgrid_fft_twiddles(g.S, false, status) : nullptr;
        if (*status) break;
        if (stw)
        {
            sdp_es::SubgridCut cut;
            cut.grid = (const float2*)(const void*)d_grid;
            cut.G = (int)G;
            cut.task = p.task;
            cut.nv = (int)g.nv;
            cut.min_iu = (int)g.min_iu;
            cut.min_iv = (int)g.min_iv;
            cut.eff = g.eff;
            cut.perm_shift = perm_n2 ? __builtin_ctz((unsigned)perm_n2) : -1;
            const int e = sdp_es::subgrid_fft2d((float*)d_wimg, g.S, gr.slots,
                    false, *stw, &cut, 0);
            if (e) *status = (sdp_Error)e;
        }
        else
        {
            const int nbx = (g.S + 255) / 256;
            k_cut_out<T><<<dim3((unsigned)(gr.slots_alloc * nbx),
                    (unsigned)((g.S + kCutRows - 1) / kCutRows)), 256>>>(d_grid, G, d_wimg, g.S, layer,
                    p.task, g.nv, g.min_iu, g.min_iv, g.eff, gr.slots, nbx,
                    perm_n2);
            sdp_fft::exec_2d(sp, d_wimg, false, 0, status);
        }
        const int64_t first = gr.first_p + g.P0 - p.off_w;
        const int64_t last = gr.last_p + g.P0 - p.off_w;
        if (g.fused)
        {
            if constexpr (sizeof(T) == 4)
            {
                // The cut-out's checkerboard and 1 / S^2 are applied as
                // k_tower_idft reads the sub-grid image (no separate pass).
                DftParams dp = {};
                dp.norm = (float)norm;
                dp.tp = p;
                dp.vrec = dd.vrec;
                dp.seg_start = dd.seg_start;
                dp.seg_end = dd.seg_end;
                dp.gslot_base = (int64_t)gi * b.t_cap;
                dp.P0 = g.P0;
                dp.wp = wp;
                dp.wp_inv = dd.wp_inv;
                dp.w_turns = dd.w_turns;
                dp.prep = dd.prep;
                dp.prep_stride = dd.prep_stride;
                dp.uv_kernel = k->d_uv_kernel;
                dp.w_kernel = k->d_w_kernel;
                dp.tw = dd.tw;
                dp.in = (const Cx<float>*)d_wimg;
                dp.part = d_part;
                tower_timing().start();
                if (two)
                    k_tower_idft<U, 2><<<dim3(ntiles, (unsigned)gr.slots),
                            256, g.S * sizeof(float2)>>>(dp, d_uvw);
                else
                    k_tower_idft<U, 1><<<dim3(ntiles, (unsigned)gr.slots),
                            256, g.S * sizeof(float2)>>>(dp, d_uvw);
                SDP_HIP_CHECK_LAUNCH(status);
                tower_timing().stop();
            }
            tm.layers += (last - first + ws_n) * gr.slots;
            if (verbosity > 0)
            {
                (void)hipDeviceSynchronize();
                tm.towers += now_s() - tg;
            }
            continue;
        }
        k_degrid_init<T><<<blocks_of(n_el), 256>>>(d_wimg, wp, layer, g.S,
                norm, (int)(first - ws_n / 2), n_el);
        for (int i = 0; i < ws_n && !*status; ++i)
        {
            k_degrid_step<T><<<blocks_of(n_el), 256>>>(d_wimg,
                    d_stack + i * ls, wp, layer, g.S, n_el);
            sdp_fft::exec_2d(sp, d_stack + i * ls, true, 0, status);
        }
        int ring = 0;
        for (int64_t w_plane = first; w_plane <= last && !*status; ++w_plane)
        {
            if (w_plane != first)
            {
                const int slot_layer = ring;
                ring = (ring + 1) % ws_n;
                k_degrid_step<T><<<blocks_of(n_el), 256>>>(d_wimg,
                        d_stack + slot_layer * ls, wp, layer, g.S, n_el);
                sdp_fft::exec_2d(sp, d_stack + slot_layer * ls, true, 0,
                        status);
            }
            const int64_t prel = w_plane + p.off_w - g.P0;
            const int64_t i0 = b.offsets[gi * (g.NP + 1) + prel];
            const int64_t i1 = b.offsets[gi * (g.NP + 1) + prel + 1];
            if (i1 > i0)
            {
                p.w_plane = (int)w_plane;
                p.ring = ring;
                k_tower_degrid<T, U><<<blocks_of(i1 - i0, kWaves),
                        64 * kWaves>>>(p, b.items + i0, i1 - i0, d_uvw,
                        d_stack, k->d_uv_kernel, k->d_w_kernel, d_vis);
            }
            SDP_HIP_CHECK_LAUNCH(status);
        }
        tm.layers += (last - first + 1) * gr.slots;
        if (verbosity > 0)
        {
            (void)hipDeviceSynchronize();
            tm.towers += now_s() - tg;
        }
    }
    if (g.fused && d_part && !*status && dd.n_vis > 0)
    {
        if constexpr (sizeof(T) == 4)
        {
            k_idft_reduce<<<blocks_of(dd.n_vis), 256>>>(dd.vrec, dd.n_vis,
                    d_part, ntiles, g.num_chan, (Cx<float>*)d_vis);
            SDP_HIP_CHECK_LAUNCH(status);
        }
    }
    if (tower_timing().on && g.fused)
    {
        TowerTiming& tt = tower_timing();
        tt.collect();
        tt.vis += dd.n_vis;
        tt.layers += tm.layers;
        tt.S = g.S;
        tt.kind = 1;
    }
    if (verbosity > 0 && !*status)
    {
        SDP_LOG_INFO("w-stacking with w-towers (degridding): %lld w-stack "
                "planes, %lld sub-grids x %lld, %zu sub-grid groups, %lld "
                "visibility runs, %lld sub-grid w-layers",
                (long long)g.niw, (long long)g.nu, (long long)g.nv,
                b.groups.size(), (long long)b.n_items, (long long)tm.layers);
        SDP_LOG_INFO("| binning %.3f s | towers %.3f s | image side %.3f s"
                " | %s", tm.bin, tm.towers, tm.image, g.fused ?
                "fused towers (k_tower_idft)" : "layer-by-layer towers");
    }
}

// Argument checks shared by grid_all and degrid_all (.cpp:241-259).
bool check_args(const sdp_Mem* vis, const sdp_Mem* uvw, const sdp_Mem* image,
        int subgrid_size, double w_tower_height, int plane_offset,
        int plane_stride, sdp_Error* status)
{
    if (*status) return false;
    const sdp_MemLocation loc = sdp_mem_location(vis);
    if (sdp_mem_location(image) != loc || sdp_mem_location(uvw) != loc)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("All arrays must be in the same memory space");
        return false;
    }
    if (sdp_mem_num_dims(vis) != 2 || sdp_mem_num_dims(uvw) != 2)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Visibilities and (u,v,w)-coordinates must be 2D");
        return false;
    }
    if (w_tower_height == 0.0)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Automatic w-tower height not yet implemented");
        return false;
    }
    if (sdp_mem_shape_dim(uvw, 1) != 3 ||
            sdp_mem_shape_dim(uvw, 0) != sdp_mem_shape_dim(vis, 0) ||
            sdp_mem_num_dims(image) != 2 ||
            sdp_mem_shape_dim(image, 0) != sdp_mem_shape_dim(image, 1) ||
            !sdp_mem_is_c_contiguous(vis) || !sdp_mem_is_c_contiguous(uvw) ||
            !sdp_mem_is_c_contiguous(image) || subgrid_size <= 0 ||
            subgrid_size % 2 != 0 ||
            subgrid_size > sdp_mem_shape_dim(image, 0) || plane_stride < 1 ||
            plane_offset < 0 || plane_offset >= plane_stride)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Inconsistent arguments: uvw must be [rows, 3], vis "
                "[rows, chans], the image square and at least the (even) "
                "sub-grid size, all C-contiguous");
        return false;
    }
    if (sdp_mem_shape_dim(vis, 0) > 0x7FFFFFFF ||
            sdp_mem_shape_dim(vis, 1) > 0x7FFFFFFF ||
            sdp_mem_shape_dim(image, 0) >= (1 << 22))
    {
        // 32-bit row / sub-grid index arithmetic in the grid kernels.
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Too many rows / channels, or image of 2^22 pixels "
                "or more a side");
        return false;
    }
    const sdp_MemType tv = sdp_mem_type(vis), tu = sdp_mem_type(uvw);
    const bool ok = (tv == SDP_MEM_COMPLEX_DOUBLE && tu == SDP_MEM_DOUBLE) ||
            (tv == SDP_MEM_COMPLEX_FLOAT && tu == SDP_MEM_DOUBLE) ||
            (tv == SDP_MEM_COMPLEX_FLOAT && tu == SDP_MEM_FLOAT);
    if (!ok || any_kind(sdp_mem_type(image)) < 0)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data types: vis %s, uvw %s, image %s",
                sdp_mem_type_name(tv), sdp_mem_type_name(tu),
                sdp_mem_type_name(sdp_mem_type(image)));
        return false;
    }
    if (!sdp_hip::device_available())
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("No GPU available for the w-towers driver.");
        return false;
    }
    return true;
}

Geo make_geo(const sdp_Mem* vis, double f0, double df, int S, double theta,
        double w_step, int support, int w_support, double subgrid_frac,
        double H, int plane_offset, int plane_stride)
{
    Geo g = {};
    g.f0 = f0;
    g.df = df;
    g.num_rows = sdp_mem_shape_dim(vis, 0);
    g.num_chan = sdp_mem_shape_dim(vis, 1);
    g.S = S;
    if (subgrid_frac == 0.0) subgrid_frac = 2.0 / 3.0;
    g.eff = int(floor(S * subgrid_frac));
    g.support = support;
    g.w_support = w_support;
    g.theta = theta;
    g.w_step = w_step;
    g.H = H;
    g.eff_dist = g.eff / theta;
    g.ws_dist = H * w_step;
    g.plane_offset = plane_offset;
    g.plane_stride = plane_stride;
    return g;
}

template<typename U>
const U* cptr(const sdp_Mem* m)
{
    return (const U*)sdp_mem_data_const(m);
}

// Plane set of the *_plane_set extension: a 1-D int32 mask, host or device
// (staged), or NULL (offset / stride selection).
bool check_mask(const sdp_Mem* mask, sdp_Error* status)
{
    if (*status || !mask) return !*status;
    if (sdp_mem_type(mask) != SDP_MEM_INT || sdp_mem_num_dims(mask) != 1 ||
            !sdp_mem_is_c_contiguous(mask))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("The plane mask must be a 1-D contiguous int32 array");
        return false;
    }
    return true;
}

void set_mask(Geo& g, const Staged& sm, int64_t first, const sdp_Mem* mask)
{
    if (!mask) return;
    g.plane_mask = (const int*)sdp_mem_data_const(sm.dev);
    g.mask_first = first;
    g.mask_n = sdp_mem_shape_dim(mask, 0);
}

void run_grid(const sdp_Mem* vis, double f0, double df, const sdp_Mem* uvw,
        int S, double theta, double w_step, double hu, double hv,
        int support, int os, int w_support, int wos, double frac, double H,
        int verbosity, sdp_Mem* image, int plane_offset, int plane_stride,
        int64_t mask_first, const sdp_Mem* mask, sdp_Error* status)
{
    if (!check_args(vis, uvw, image, S, H, plane_offset, plane_stride,
            status) || !check_mask(mask, status))
        return;
    std::lock_guard<std::mutex> lock(g_mutex);
    const int64_t G = sdp_mem_shape_dim(image, 0);
    sdp_GridderWtowerUVW* k = cached_kernel((int)G, S, theta, w_step, hu, hv,
            support, os, w_support, wos, status);
    if (*status) return;
    Staged sv, su, si, sm;
    sv.init(vis, status);
    su.init(uvw, status);
    si.init(image, status);
    if (mask) sm.init(mask, status);
    if (*status) return;
    // Output image cleared first (.cpp:604-606).
    SDP_HIP_CHECK(hipMemsetAsync(sdp_mem_data(si.dev), 0,
            sdp_mem_num_elements(image) *
            sdp_mem_type_size(sdp_mem_type(image)), 0), status);
    Geo g = make_geo(vis, f0, df, S, theta, w_step, support, w_support, frac,
            H, plane_offset, plane_stride);
    set_mask(g, sm, mask_first, mask);
    const AnyView img = {sdp_mem_data(si.dev),
            any_kind(sdp_mem_type(image))};
    const sdp_MemType tv = sdp_mem_type(vis), tu = sdp_mem_type(uvw);
    if (g.num_rows > 0 && g.num_chan > 0)
    {
        if (tv == SDP_MEM_COMPLEX_DOUBLE)
            grid_all_impl<double, double>(k, g,
                    cptr<Cx<double> >(sv.dev), cptr<double>(su.dev), img, G,
                    verbosity, status);
        else if (tu == SDP_MEM_DOUBLE)
            grid_all_impl<float, double>(k, g, cptr<Cx<float> >(sv.dev),
                    cptr<double>(su.dev), img, G, verbosity, status);
        else
            grid_all_impl<float, float>(k, g, cptr<Cx<float> >(sv.dev),
                    cptr<float>(su.dev), img, G, verbosity, status);
    }
    si.write_back(status);
}

void run_degrid(const sdp_Mem* image, double f0, double df,
        const sdp_Mem* uvw, int S, double theta, double w_step, double hu,
        double hv, int support, int os, int w_support, int wos, double frac,
        double H, int verbosity, sdp_Mem* vis, int plane_offset,
        int plane_stride, int64_t mask_first, const sdp_Mem* mask,
        sdp_Error* status)
{
    if (!check_args(vis, uvw, image, S, H, plane_offset, plane_stride,
            status) || !check_mask(mask, status))
        return;
    std::lock_guard<std::mutex> lock(g_mutex);
    const int64_t G = sdp_mem_shape_dim(image, 0);
    sdp_GridderWtowerUVW* k = cached_kernel((int)G, S, theta, w_step, hu, hv,
            support, os, w_support, wos, status);
    if (*status) return;
    Staged sv, su, si, sm;
    sv.init(vis, status);
    su.init(uvw, status);
    si.init(image, status);
    if (mask) sm.init(mask, status);
    if (*status) return;
    // Output visibilities cleared first (.cpp:332-334).
    SDP_HIP_CHECK(hipMemsetAsync(sdp_mem_data(sv.dev), 0,
            sdp_mem_num_elements(vis) * sdp_mem_type_size(sdp_mem_type(vis)),
            0), status);
    Geo g = make_geo(vis, f0, df, S, theta, w_step, support, w_support, frac,
            H, plane_offset, plane_stride);
    set_mask(g, sm, mask_first, mask);
    const AnyView img = {sdp_mem_data(si.dev),
            any_kind(sdp_mem_type(image))};
    const sdp_MemType tv = sdp_mem_type(vis), tu = sdp_mem_type(uvw);
    if (g.num_rows > 0 && g.num_chan > 0)
    {
        if (tv == SDP_MEM_COMPLEX_DOUBLE)
            degrid_all_impl<double, double>(k, g, img, G,
                    cptr<double>(su.dev), (Cx<double>*)sdp_mem_data(sv.dev),
                    verbosity, status);
        else if (tu == SDP_MEM_DOUBLE)
            degrid_all_impl<float, double>(k, g, img, G,
                    cptr<double>(su.dev), (Cx<float>*)sdp_mem_data(sv.dev),
                    verbosity, status);
        else
            degrid_all_impl<float, float>(k, g, img, G, cptr<float>(su.dev),
                    (Cx<float>*)sdp_mem_data(sv.dev), verbosity, status);
    }
    sv.write_back(status);
}

} // namespace

extern "C" {

void sdp_grid_wstack_wtower_grid_all(const sdp_Mem* vis, double freq0_hz,
        double dfreq_hz, const sdp_Mem* uvw, int subgrid_size, double theta,
        double w_step, double shear_u, double shear_v, int support,
        int oversampling, int w_support, int w_oversampling,
        double subgrid_frac, double w_tower_height, int verbosity,
        sdp_Mem* image, int num_threads, sdp_Error* status)
{
    (void)num_threads;
    run_grid(vis, freq0_hz, dfreq_hz, uvw, subgrid_size, theta, w_step,
            shear_u, shear_v, support, oversampling, w_support,
            w_oversampling, subgrid_frac, w_tower_height, verbosity, image, 0,
            1, 0, nullptr, status);
}

void sdp_grid_wstack_wtower_degrid_all(const sdp_Mem* image,
        double freq0_hz, double dfreq_hz, const sdp_Mem* uvw,
        int subgrid_size, double theta, double w_step, double shear_u,
        double shear_v, int support, int oversampling, int w_support,
        int w_oversampling, double subgrid_frac, double w_tower_height,
        int verbosity, sdp_Mem* vis, int num_threads, sdp_Error* status)
{
    (void)num_threads;
    run_degrid(image, freq0_hz, dfreq_hz, uvw, subgrid_size, theta, w_step,
            shear_u, shear_v, support, oversampling, w_support,
            w_oversampling, subgrid_frac, w_tower_height, verbosity, vis, 0,
            1, 0, nullptr, status);
}

void sdp_grid_wstack_wtower_grid_planes(const sdp_Mem* vis, double freq0_hz,
        double dfreq_hz, const sdp_Mem* uvw, int subgrid_size, double theta,
        double w_step, double shear_u, double shear_v, int support,
        int oversampling, int w_support, int w_oversampling,
        double subgrid_frac, double w_tower_height, int verbosity,
        sdp_Mem* image, int plane_offset, int plane_stride, sdp_Error* status)
{
    run_grid(vis, freq0_hz, dfreq_hz, uvw, subgrid_size, theta, w_step,
            shear_u, shear_v, support, oversampling, w_support,
            w_oversampling, subgrid_frac, w_tower_height, verbosity, image,
            plane_offset, plane_stride, 0, nullptr, status);
}

void sdp_grid_wstack_wtower_grid_plane_set(const sdp_Mem* vis,
        double freq0_hz, double dfreq_hz, const sdp_Mem* uvw,
        int subgrid_size, double theta, double w_step, double shear_u,
        double shear_v, int support, int oversampling, int w_support,
        int w_oversampling, double subgrid_frac, double w_tower_height,
        int verbosity, sdp_Mem* image, int64_t plane_first,
        const sdp_Mem* plane_mask, sdp_Error* status)
{
    if (!plane_mask && !*status)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("No plane mask given");
        return;
    }
    run_grid(vis, freq0_hz, dfreq_hz, uvw, subgrid_size, theta, w_step,
            shear_u, shear_v, support, oversampling, w_support,
            w_oversampling, subgrid_frac, w_tower_height, verbosity, image,
            0, 1, plane_first, plane_mask, status);
}

void sdp_grid_wstack_wtower_degrid_planes(const sdp_Mem* image,
        double freq0_hz, double dfreq_hz, const sdp_Mem* uvw,
        int subgrid_size, double theta, double w_step, double shear_u,
        double shear_v, int support, int oversampling, int w_support,
        int w_oversampling, double subgrid_frac, double w_tower_height,
        int verbosity, sdp_Mem* vis, int plane_offset, int plane_stride,
        sdp_Error* status)
{
    run_degrid(image, freq0_hz, dfreq_hz, uvw, subgrid_size, theta, w_step,
            shear_u, shear_v, support, oversampling, w_support,
            w_oversampling, subgrid_frac, w_tower_height, verbosity, vis,
            plane_offset, plane_stride, 0, nullptr, status);
}

void sdp_grid_wstack_wtower_degrid_plane_set(const sdp_Mem* image,
        double freq0_hz, double dfreq_hz, const sdp_Mem* uvw,
        int subgrid_size, double theta, double w_step, double shear_u,
        double shear_v, int support, int oversampling, int w_support,
        int w_oversampling, double subgrid_frac, double w_tower_height,
        int verbosity, sdp_Mem* vis, int64_t plane_first,
        const sdp_Mem* plane_mask, sdp_Error* status)
{
    if (!plane_mask && !*status)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("No plane mask given");
        return;
    }
    run_degrid(image, freq0_hz, dfreq_hz, uvw, subgrid_size, theta, w_step,
            shear_u, shear_v, support, oversampling, w_support,
            w_oversampling, subgrid_frac, w_tower_height, verbosity, vis,
            0, 1, plane_first, plane_mask, status);
}

void sdp_grid_wstack_wtower_enable_timing(int enable)
{
    TowerTiming& tt = tower_timing();
    tt.collect();
    tt.on = enable != 0;
    tt.ms = 0;
    tt.launches = tt.vis = tt.layers = 0;
    tt.S = tt.kind = 0;
}

int sdp_grid_wstack_wtower_get_timing(double* out, int max_values)
{
    TowerTiming& tt = tower_timing();
    if (!tt.on || !out) return 0;
    tt.collect();
    const double v[6] = {tt.ms, (double)tt.launches, (double)tt.vis,
            (double)tt.layers, (double)tt.S, (double)tt.kind};
    const int n = max_values < 6 ? max_values : 6;
    for (int i = 0; i < n; ++i) out[i] = v[i];
    return n;
}

} // extern "C"
