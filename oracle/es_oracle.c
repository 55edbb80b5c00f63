/*
 * TEST INFRASTRUCTURE ONLY -- CPU oracle for the ES (de)gridding hot path.
 *
 * This file is a plain-C restatement of the per-visibility arithmetic of the
 * reference CUDA kernels, used by tests/, __graft_entry__.smoke() and the
 * bench.py cpu_baseline leg as the CHECKER. It is never linked into, loaded
 * by or called from the product library (ska-sdp-func_amd/).
 *
 * Reference followed (ska-sdp-func 1.2.2):
 *   src/ska-sdp-func/grid_data/sdp_gridder_uvw_es_fft_kernels.cu
 *     exp_semicircle            :97-102
 *     gridding_3d (grid/degrid) :126-270   (w<0 flip + conjugate :158,167,268)
 *     gridding_2d (grid/degrid) :277-422
 *
 * Precision policy: the coordinate / tap arithmetic is done in the SAME
 * precision and operation order as the reference kernel (float for the f32
 * path, double for the f64 path), so the oracle sees exactly the taps the
 * reference would use. Accumulation is done in double ("expected value" of the
 * reference's order-dependent float atomics).
 *
 * Grid layout: complex, row-major [G][G], index (u + G/2) * G + (v + G/2)
 * (u is the slow / row axis: kernels.cu:238-240, 390-392).
 */
#include <math.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define C_LIGHT 299792458.0

/* Threads of the OpenMP loops below (the bench's CPU baseline sets the
 * job's CPU share; returns the count in effect). */
int oracle_set_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

/* ---- f32 path ---------------------------------------------------------- */

static inline float es_f(float beta, float x)
{
    /* kernels.cu:97-102 */
    const float xx = x * x;
    return (xx > 1.0f) ? 0.0f : expf(beta * (sqrtf(1.0f - xx) - 1.0f));
}

static inline double es_d(double beta, double x)
{
    const double xx = x * x;
    return (xx > 1.0) ? 0.0 : exp(beta * (sqrt(1.0 - xx) - 1.0));
}

/*
 * Visit every tap of one visibility, f32 arithmetic.
 * mode 0: grid   -> grid_acc (double complex, interleaved) += w*V*k
 * mode 1: degrid -> returns sum over taps of grid_in * k (double accumulate)
 * plane: the single w-plane index being processed (3-D), ignored if !do_w.
 */
static void visit_f32(
        int do_w, int mode, int G, int support, float beta, float uv_scale,
        float w_scale, float min_plane_w, int plane,
        const float* uvw_row, float freq, const float vis_w[2],
        double* grid_acc, const double* grid_in, double out[2],
        int row_lo, int row_hi)
{
    const float flip = do_w ? ((uvw_row[2] < 0.0f) ? -1.0f : 1.0f) : 1.0f;
    const float inv_wavelength = flip * freq / (float)C_LIGHT;
    const float half_support = (float)support / 2.0f;
    const int grid_min_uv = -G / 2;
    const int grid_max_uv = (G - 1) / 2;
    const float pos_u = uvw_row[0] * inv_wavelength * uv_scale;
    const float pos_v = uvw_row[1] * inv_wavelength * uv_scale;
    const float pos_w = do_w ?
            (uvw_row[2] * inv_wavelength - min_plane_w) * w_scale : 0.0f;
    int u_min = (int)ceilf(pos_u - half_support);
    int u_max = (int)floorf(pos_u + half_support);
    int v_min = (int)ceilf(pos_v - half_support);
    int v_max = (int)floorf(pos_v + half_support);
    int w_min = (int)ceilf(pos_w - half_support);
    int w_max = (int)floorf(pos_w + half_support);
    if (u_min < grid_min_uv) u_min = grid_min_uv;
    if (u_max > grid_max_uv) u_max = grid_max_uv;
    if (v_min < grid_min_uv) v_min = grid_min_uv;
    if (v_max > grid_max_uv) v_max = grid_max_uv;
    if (w_min < plane) w_min = plane;
    if (w_max > plane) w_max = plane;
    out[0] = out[1] = 0.0;
    if (w_min > w_max || u_min > u_max || v_min > v_max) return;
    const float inv_hs = 1.0f / half_support;
    float ku[64], kv[64];
    for (int u = u_min; u <= u_max; ++u)
        ku[u - u_min] = es_f(beta, ((float)u - pos_u) * inv_hs);
    for (int v = v_min; v <= v_max; ++v)
        kv[v - v_min] = es_f(beta, ((float)v - pos_v) * inv_hs);
    const float kw = es_f(beta, ((float)plane - pos_w) * inv_hs);
    const float vre = vis_w[0], vim = vis_w[1] * flip;
    double acc_re = 0.0, acc_im = 0.0;
    const int off = G / 2;
    for (int u = u_min; u <= u_max; ++u)
    {
        if (u < row_lo || u > row_hi) continue;
        for (int v = v_min; v <= v_max; ++v)
        {
            float k = ku[u - u_min] * kv[v - v_min] * kw;
            if ((u + v) & 1) k = -k;
            const size_t idx = (size_t)(u + off) * G + (size_t)(v + off);
            if (mode == 0)
            {
                grid_acc[2 * idx] += (double)(vre * k);
                grid_acc[2 * idx + 1] += (double)(vim * k);
            }
            else
            {
                acc_re += grid_in[2 * idx] * (double)k;
                acc_im += grid_in[2 * idx + 1] * (double)k;
            }
        }
    }
    out[0] = acc_re;
    out[1] = acc_im * (double)flip;   /* kernels.cu:267-268 */
}

static void visit_f64(
        int do_w, int mode, int G, int support, double beta, double uv_scale,
        double w_scale, double min_plane_w, int plane,
        const double* uvw_row, double freq, const double vis_w[2],
        double* grid_acc, const double* grid_in, double out[2],
        int row_lo, int row_hi)
{
    const double flip = do_w ? ((uvw_row[2] < 0.0) ? -1.0 : 1.0) : 1.0;
    const double inv_wavelength = flip * freq / C_LIGHT;
    const double half_support = (double)support / 2.0;
    const int grid_min_uv = -G / 2;
    const int grid_max_uv = (G - 1) / 2;
    const double pos_u = uvw_row[0] * inv_wavelength * uv_scale;
    const double pos_v = uvw_row[1] * inv_wavelength * uv_scale;
    const double pos_w = do_w ?
            (uvw_row[2] * inv_wavelength - min_plane_w) * w_scale : 0.0;
    int u_min = (int)ceil(pos_u - half_support);
    int u_max = (int)floor(pos_u + half_support);
    int v_min = (int)ceil(pos_v - half_support);
    int v_max = (int)floor(pos_v + half_support);
    int w_min = (int)ceil(pos_w - half_support);
    int w_max = (int)floor(pos_w + half_support);
    if (u_min < grid_min_uv) u_min = grid_min_uv;
    if (u_max > grid_max_uv) u_max = grid_max_uv;
    if (v_min < grid_min_uv) v_min = grid_min_uv;
    if (v_max > grid_max_uv) v_max = grid_max_uv;
    if (w_min < plane) w_min = plane;
    if (w_max > plane) w_max = plane;
    out[0] = out[1] = 0.0;
    if (w_min > w_max || u_min > u_max || v_min > v_max) return;
    const double inv_hs = 1.0 / half_support;
    double ku[64], kv[64];
    for (int u = u_min; u <= u_max; ++u)
        ku[u - u_min] = es_d(beta, ((double)u - pos_u) * inv_hs);
    for (int v = v_min; v <= v_max; ++v)
        kv[v - v_min] = es_d(beta, ((double)v - pos_v) * inv_hs);
    const double kw = es_d(beta, ((double)plane - pos_w) * inv_hs);
    const double vre = vis_w[0], vim = vis_w[1] * flip;
    double acc_re = 0.0, acc_im = 0.0;
    const int off = G / 2;
    for (int u = u_min; u <= u_max; ++u)
    {
        if (u < row_lo || u > row_hi) continue;
        for (int v = v_min; v <= v_max; ++v)
        {
            double k = ku[u - u_min] * kv[v - v_min] * kw;
            if ((u + v) & 1) k = -k;
            const size_t idx = (size_t)(u + off) * G + (size_t)(v + off);
            if (mode == 0)
            {
                grid_acc[2 * idx] += vre * k;
                grid_acc[2 * idx + 1] += vim * k;
            }
            else
            {
                acc_re += grid_in[2 * idx] * k;
                acc_im += grid_in[2 * idx + 1] * k;
            }
        }
    }
    out[0] = acc_re;
    out[1] = acc_im * flip;
}

/*
 * Scatter all visibilities onto one w-plane (2-D: plane 0, do_w 0).
 * vis: interleaved complex [R][C]; weight [R][C]; uvw [R][3]; freq [C];
 * grid: double complex interleaved [G][G], accumulated into (not cleared).
 * Weighting: vis * weight in working precision (kernels.cu:163-167).
 */
void oracle_es_grid_f32(
        int64_t num_rows, int num_chan, const float* uvw, const float* freq,
        const float* vis, const float* weight, int G, int support,
        float beta, float uv_scale, float w_scale, float min_plane_w,
        int do_w, int plane, double* grid)
{
    for (int64_t r = 0; r < num_rows; ++r)
    {
        for (int c = 0; c < num_chan; ++c)
        {
            const int64_t i = r * num_chan + c;
            float vw[2] = { vis[2 * i] * weight[i], vis[2 * i + 1] * weight[i] };
            double dummy[2];
            visit_f32(do_w, 0, G, support, beta, uv_scale, w_scale,
                    min_plane_w, plane, uvw + 3 * r, freq[c], vw, grid, 0,
                    dummy, INT32_MIN, INT32_MAX);
        }
    }
}

void oracle_es_grid_f64(
        int64_t num_rows, int num_chan, const double* uvw,
        const double* freq, const double* vis, const double* weight, int G,
        int support, double beta, double uv_scale, double w_scale,
        double min_plane_w, int do_w, int plane, double* grid)
{
    for (int64_t r = 0; r < num_rows; ++r)
    {
        for (int c = 0; c < num_chan; ++c)
        {
            const int64_t i = r * num_chan + c;
            double vw[2] = { vis[2 * i] * weight[i], vis[2 * i + 1] * weight[i] };
            double dummy[2];
            visit_f64(do_w, 0, G, support, beta, uv_scale, w_scale,
                    min_plane_w, plane, uvw + 3 * r, freq[c], vw, grid, 0,
                    dummy, INT32_MIN, INT32_MAX);
        }
    }
}

/*
 * Gather from one w-plane: out_vis (double complex [R][C]) += taps * grid.
 * Weights are NOT applied in degridding (kernels.cu:169-172, 320-323).
 */
void oracle_es_degrid_f32(
        int64_t num_rows, int num_chan, const float* uvw, const float* freq,
        const double* grid, int G, int support, float beta, float uv_scale,
        float w_scale, float min_plane_w, int do_w, int plane,
        double* out_vis)
{
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < num_rows; ++r)
    {
        for (int c = 0; c < num_chan; ++c)
        {
            const int64_t i = r * num_chan + c;
            const float zero[2] = { 0.0f, 0.0f };
            double o[2];
            visit_f32(do_w, 1, G, support, beta, uv_scale, w_scale,
                    min_plane_w, plane, uvw + 3 * r, freq[c], zero, 0, grid,
                    o, INT32_MIN, INT32_MAX);
            out_vis[2 * i] += o[0];
            out_vis[2 * i + 1] += o[1];
        }
    }
}

void oracle_es_degrid_f64(
        int64_t num_rows, int num_chan, const double* uvw,
        const double* freq, const double* grid, int G, int support,
        double beta, double uv_scale, double w_scale, double min_plane_w,
        int do_w, int plane, double* out_vis)
{
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < num_rows; ++r)
    {
        for (int c = 0; c < num_chan; ++c)
        {
            const int64_t i = r * num_chan + c;
            const double zero[2] = { 0.0, 0.0 };
            double o[2];
            visit_f64(do_w, 1, G, support, beta, uv_scale, w_scale,
                    min_plane_w, plane, uvw + 3 * r, freq[c], zero, 0, grid,
                    o, INT32_MIN, INT32_MAX);
            out_vis[2 * i] += o[0];
            out_vis[2 * i + 1] += o[1];
        }
    }
}

/*
 * Same result as oracle_es_grid_f32 / _f64 (identical taps, double
 * accumulation, each cell's contributions summed in visibility order), but
 * multi-threaded for the full-size parity tests: grid rows are split into
 * stripes, visibilities are binned by the stripes their u taps touch, and
 * each stripe is accumulated by one thread restricted to its rows.
 */
#define U_SPAN(FT, CEIL, FLOOR)                                              \
    const FT flip = do_w ? ((uvw[3 * r + 2] < (FT)0) ? (FT)-1 : (FT)1)      \
                         : (FT)1;                                            \
    const FT inv_wl = flip * freq[c] / (FT)C_LIGHT;                          \
    const FT hs = (FT)support / (FT)2;                                       \
    const FT pu = uvw[3 * r] * inv_wl * uv_scale;                            \
    const FT pw = do_w ? (uvw[3 * r + 2] * inv_wl - min_plane_w) * w_scale   \
                       : (FT)0;                                              \
    int u0 = (int)CEIL(pu - hs), u1 = (int)FLOOR(pu + hs);                   \
    int w0 = (int)CEIL(pw - hs), w1 = (int)FLOOR(pw + hs);                   \
    if (u0 < -(G / 2)) u0 = -(G / 2);                                        \
    if (u1 > (G - 1) / 2) u1 = (G - 1) / 2;                                  \
    if (w0 < plane) w0 = plane;                                              \
    if (w1 > plane) w1 = plane;                                              \
    const int skip = (w0 > w1 || u0 > u1);

#define GRID_PAR(NAME, FT, VISIT, CEIL, FLOOR)                               \
int NAME(int64_t num_rows, int num_chan, const FT* uvw, const FT* freq,      \
        const FT* vis, const FT* weight, int G, int support, FT beta,        \
        FT uv_scale, FT w_scale, FT min_plane_w, int do_w, int plane,        \
        double* grid)                                                        \
{                                                                            \
    int nth = 1;                                                             \
    _OMP_MAXTHREADS(nth);                                                    \
    const int64_t nvis = num_rows * num_chan;                                \
    const int ns = 4 * nth;                                                  \
    const int rows_per = (G + ns - 1) / ns;                                  \
    const int off = G / 2;                                                   \
    int64_t* cnt = (int64_t*)calloc((size_t)nth * ns, sizeof(int64_t));      \
    int64_t* start = (int64_t*)calloc((size_t)ns + 1, sizeof(int64_t));      \
    if (!cnt || !start) return -1;                                           \
    _Pragma("omp parallel")                                                  \
    {                                                                        \
        int tid = 0;                                                         \
        _OMP_TID(tid);                                                       \
        int64_t* my = cnt + (size_t)tid * ns;                                \
        _Pragma("omp for schedule(static)")                                  \
        for (int64_t i = 0; i < nvis; ++i)                                   \
        {                                                                    \
            const int64_t r = i / num_chan;                                  \
            const int c = (int)(i - r * num_chan);                           \
            U_SPAN(FT, CEIL, FLOOR)                                          \
            if (skip) continue;                                              \
            for (int s = (u0 + off) / rows_per; s <= (u1 + off) / rows_per;  \
                    ++s)                                                     \
                my[s]++;                                                     \
        }                                                                    \
    }                                                                        \
    int64_t total = 0;                                                       \
    for (int s = 0; s < ns; ++s)                                             \
    {                                                                        \
        start[s] = total;                                                    \
        for (int t = 0; t < nth; ++t)                                        \
        {                                                                    \
            const int64_t n = cnt[(size_t)t * ns + s];                       \
            cnt[(size_t)t * ns + s] = total;                                 \
            total += n;                                                      \
        }                                                                    \
    }                                                                        \
    start[ns] = total;                                                       \
    int64_t* list = (int64_t*)malloc((size_t)(total > 0 ? total : 1) *      \
            sizeof(int64_t));                                                \
    if (!list) return -1;                                                    \
    _Pragma("omp parallel")                                                  \
    {                                                                        \
        int tid = 0;                                                         \
        _OMP_TID(tid);                                                       \
        int64_t* my = cnt + (size_t)tid * ns;                                \
        _Pragma("omp for schedule(static)")                                  \
        for (int64_t i = 0; i < nvis; ++i)                                   \
        {                                                                    \
            const int64_t r = i / num_chan;                                  \
            const int c = (int)(i - r * num_chan);                           \
            U_SPAN(FT, CEIL, FLOOR)                                          \
            if (skip) continue;                                              \
            for (int s = (u0 + off) / rows_per; s <= (u1 + off) / rows_per;  \
                    ++s)                                                     \
                list[my[s]++] = i;                                           \
        }                                                                    \
    }                                                                        \
    _Pragma("omp parallel for schedule(dynamic, 1)")                         \
    for (int s = 0; s < ns; ++s)                                             \
    {                                                                        \
        const int lo = s * rows_per - off, hi = lo + rows_per - 1;           \
        for (int64_t e = start[s]; e < start[s + 1]; ++e)                    \
        {                                                                    \
            const int64_t i = list[e];                                       \
            const int64_t r = i / num_chan;                                  \
            const int c = (int)(i - r * num_chan);                           \
            FT vw[2] = { vis[2 * i] * weight[i], vis[2 * i + 1] * weight[i] };\
            double dummy[2];                                                 \
            VISIT(do_w, 0, G, support, beta, uv_scale, w_scale, min_plane_w, \
                    plane, uvw + 3 * r, freq[c], vw, grid, 0, dummy, lo, hi);\
        }                                                                    \
    }                                                                        \
    free(list);                                                              \
    free(start);                                                             \
    free(cnt);                                                               \
    return nth;                                                              \
}

#ifdef _OPENMP
#define _OMP_MAXTHREADS(n) (n) = omp_get_max_threads()
#define _OMP_TID(t) (t) = omp_get_thread_num()
#else
#define _OMP_MAXTHREADS(n) (void)(n)
#define _OMP_TID(t) (void)(t)
#endif

GRID_PAR(oracle_es_grid_f32_par, float, visit_f32, ceilf, floorf)
GRID_PAR(oracle_es_grid_f64_par, double, visit_f64, ceil, floor)

/*
 * CPU baseline leg (bench.py only): a multi-threaded CPU gridder of the
 * reference's f32 arithmetic (same taps as visit_f32). Grid rows are split
 * into stripes; visibilities are binned by the stripes their taps touch
 * (counting sort, per-thread counts), then threads take whole stripes, so
 * every grid cell is written by one thread: no private grids, no atomics.
 * Accumulates into grid_out (complex64, interleaved). Returns the number of
 * OpenMP threads used.
 */
int oracle_es_grid_f32_omp(
        int64_t num_rows, int num_chan, const float* uvw, const float* freq,
        const float* vis, const float* weight, int G, int support,
        float beta, float uv_scale, float* grid_out)
{
    int nthreads = 1;
#ifdef _OPENMP
    nthreads = omp_get_max_threads();
#endif
    const int64_t nvis = num_rows * num_chan;
    const int nstripes = 8 * nthreads;
    const int rows_per = (G + nstripes - 1) / nstripes;
    const float half_support = (float)support / 2.0f;
    const float inv_hs = 1.0f / half_support;
    const int off = G / 2;
    int64_t* counts = (int64_t*)calloc((size_t)nthreads * (nstripes + 1),
            sizeof(int64_t));
    if (!counts) return -1;
    /* pass 1: count (vis, stripe) entries per thread */
#pragma omp parallel
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        int64_t* my = counts + (size_t)tid * (nstripes + 1);
#pragma omp for schedule(static)
        for (int64_t i = 0; i < nvis; ++i)
        {
            const int64_t r = i / num_chan;
            const int c = (int)(i - r * num_chan);
            const float inv_wl = 1.0f * freq[c] / (float)C_LIGHT;
            const float pu = uvw[3 * r] * inv_wl * uv_scale;
            int u0 = (int)ceilf(pu - half_support);
            int u1 = (int)floorf(pu + half_support);
            if (u0 < -off) u0 = -off;
            if (u1 > (G - 1) / 2) u1 = (G - 1) / 2;
            if (u0 > u1) continue;
            for (int s = (u0 + off) / rows_per; s <= (u1 + off) / rows_per; ++s)
                my[s]++;
        }
    }
    /* prefix: stripe-major, thread-minor */
    int64_t* start = (int64_t*)calloc((size_t)nstripes + 1, sizeof(int64_t));
    int64_t total = 0;
    for (int s = 0; s < nstripes; ++s)
    {
        start[s] = total;
        for (int t = 0; t < nthreads; ++t)
        {
            const int64_t n = counts[(size_t)t * (nstripes + 1) + s];
            counts[(size_t)t * (nstripes + 1) + s] = total;
            total += n;
        }
    }
    start[nstripes] = total;
    int64_t* list = (int64_t*)malloc((size_t)(total > 0 ? total : 1) *
            sizeof(int64_t));
    /* pass 2: fill (same static schedule -> same thread/chunk mapping) */
#pragma omp parallel
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        int64_t* my = counts + (size_t)tid * (nstripes + 1);
#pragma omp for schedule(static)
        for (int64_t i = 0; i < nvis; ++i)
        {
            const int64_t r = i / num_chan;
            const int c = (int)(i - r * num_chan);
            const float inv_wl = 1.0f * freq[c] / (float)C_LIGHT;
            const float pu = uvw[3 * r] * inv_wl * uv_scale;
            int u0 = (int)ceilf(pu - half_support);
            int u1 = (int)floorf(pu + half_support);
            if (u0 < -off) u0 = -off;
            if (u1 > (G - 1) / 2) u1 = (G - 1) / 2;
            if (u0 > u1) continue;
            for (int s = (u0 + off) / rows_per; s <= (u1 + off) / rows_per; ++s)
                list[my[s]++] = i;
        }
    }
    /* pass 3: each stripe by one thread */
#pragma omp parallel for schedule(dynamic, 1)
    for (int s = 0; s < nstripes; ++s)
    {
        const int row_lo = s * rows_per - off;
        const int row_hi = row_lo + rows_per - 1;
        for (int64_t e = start[s]; e < start[s + 1]; ++e)
        {
            const int64_t i = list[e];
            const int64_t r = i / num_chan;
            const int c = (int)(i - r * num_chan);
            const float inv_wl = 1.0f * freq[c] / (float)C_LIGHT;
            const float pu = uvw[3 * r] * inv_wl * uv_scale;
            const float pv = uvw[3 * r + 1] * inv_wl * uv_scale;
            int u0 = (int)ceilf(pu - half_support);
            int u1 = (int)floorf(pu + half_support);
            int v0 = (int)ceilf(pv - half_support);
            int v1 = (int)floorf(pv + half_support);
            if (u0 < -off) u0 = -off;
            if (v0 < -off) v0 = -off;
            if (u1 > (G - 1) / 2) u1 = (G - 1) / 2;
            if (v1 > (G - 1) / 2) v1 = (G - 1) / 2;
            if (v0 > v1) continue;
            const int a0 = u0 > row_lo ? u0 : row_lo;
            const int a1 = u1 < row_hi ? u1 : row_hi;
            float kv[64];
            for (int v = v0; v <= v1; ++v)
                kv[v - v0] = es_f(beta, ((float)v - pv) * inv_hs);
            const float vre = vis[2 * i] * weight[i];
            const float vim = vis[2 * i + 1] * weight[i];
            for (int u = a0; u <= a1; ++u)
            {
                const float ku = es_f(beta, ((float)u - pu) * inv_hs);
                float* row = grid_out + 2 * ((size_t)(u + off) * G + off);
                for (int v = v0; v <= v1; ++v)
                {
                    float k = ku * kv[v - v0];
                    if ((u + v) & 1) k = -k;
                    row[2 * v] += vre * k;
                    row[2 * v + 1] += vim * k;
                }
            }
        }
    }
    free(list);
    free(start);
    free(counts);
    return nthreads;
}
