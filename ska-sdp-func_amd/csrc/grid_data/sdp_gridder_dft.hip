// Direct Fourier transforms and image helpers of the gridder utilities:
// sdp_gridder_dft / _idft / _residual / _image_to_flmn /
// _count_nonzero_pixels of include/ska-sdp-func/grid_data/
// sdp_gridder_utils.h, replacing src/ska-sdp-func/grid_data/
// sdp_gridder_utils.cpp:106-316, 429-458, 987-1013, 1042-1301, 1383-1466
// (and the idft kernel of sdp_gridder_utils.cu) of ska-sdp-func 1.2.2.
//
// These are the reference-data generators of the w-towers tests
// (test_gridder_wtower_uvw.cpp:150-254). DFT and iDFT run on the GPU with
// the reference's arithmetic: phase in double, phasor rounded to the
// visibility precision, sums in the visibility precision in the
// reference's loop order. image_to_flmn fills host (CPU) arrays, as in the
// reference. Host inputs are staged through device memory.
#include <cmath>
#include <complex>
#include <vector>

#include "ska-sdp-func/grid_data/sdp_gridder_utils.h"
#include "wtower_math.h"
#include "wtower_ops.h"
#include "../utility/sdp_hip.h"

using namespace sdp_wt;

namespace {

constexpr double kC0 = 299792458.0;
constexpr double kTwoPi = 2.0 * 3.14159265358979323846;

template<typename V>
struct C2
{
    V re, im;
};

template<typename V>
__device__ __forceinline__ C2<V> cmul2(C2<V> a, C2<V> b)
{
#pragma clang fp contract(off)
    return C2<V>{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}

// sdp_gridder_utils.cpp:126-212. One thread per (row, channel).
template<typename D, typename U, typename V>
__global__ void k_dft(const U* __restrict__ uvw, const int* start_chs,
        const int* end_chs, const double* __restrict__ flux,
        const D* __restrict__ lmn, int num_src, double du, double dv,
        double dw, double f0, double df, int64_t rows, int num_chan,
        C2<V>* __restrict__ vis)
{
#pragma clang fp contract(off)
    __shared__ double s_src[256][4];
    const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t i = k / num_chan;
    const int c = (int)(k - i * num_chan);
    bool active = i < rows;
    if (active && start_chs && end_chs && start_chs[i] >= end_chs[i])
        active = false;
    double u = 0, v = 0, w = 0;
    if (active)
    {
        const double inv_wave = (f0 + df * c) / kC0;
        u = (double)uvw[3 * i] * inv_wave - du;
        v = (double)uvw[3 * i + 1] * inv_wave - dv;
        w = (double)uvw[3 * i + 2] * inv_wave - dw;
    }
    C2<V> acc{V(0), V(0)};
    for (int s0 = 0; s0 < num_src; s0 += 256)
    {
        __syncthreads();
        const int s = s0 + (int)threadIdx.x;
        if (s < num_src)
        {
            s_src[threadIdx.x][0] = (double)lmn[3 * s];
            s_src[threadIdx.x][1] = (double)lmn[3 * s + 1];
            s_src[threadIdx.x][2] = (double)lmn[3 * s + 2];
            s_src[threadIdx.x][3] = flux[s];
        }
        __syncthreads();
        const int n = min(256, num_src - s0);
        if (!active) continue;
        for (int j = 0; j < n; ++j)
        {
            const double phase = -kTwoPi * (s_src[j][0] * u +
                    s_src[j][1] * v + s_src[j][2] * w);
            const C2<V> ph{(V)cos(phase), (V)sin(phase)};
            const C2<V> f{(V)s_src[j][3], V(0)};
            const C2<V> t = cmul2(f, ph);
            acc.re += t.re;
            acc.im += t.im;
        }
    }
    if (active)
    {
        vis[k].re += acc.re;
        vis[k].im += acc.im;
    }
}

// sdp_gridder_utils.cpp:215-314 / sdp_gridder_utils.cu idft. One thread
// per pixel s = il * image_size + im; rows and channels in order.
template<typename D, typename U, typename V>
__global__ void k_idft(const U* __restrict__ uvw, const C2<V>* __restrict__ vis,
        const int* start_chs, const int* end_chs, const D* __restrict__ lmn,
        const double* taper, double du, double dv, double dw, double f0,
        double df, int64_t rows, int num_chan, int64_t image_size,
        C2<V>* __restrict__ image)
{
#pragma clang fp contract(off)
    const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (s >= image_size * image_size) return;
    const double l = (double)lmn[3 * s], m = (double)lmn[3 * s + 1];
    const double n = (double)lmn[3 * s + 2];
    C2<V> acc{V(0), V(0)};
    for (int64_t i = 0; i < rows; ++i)
    {
        if (start_chs && end_chs && start_chs[i] >= end_chs[i]) continue;
        const double x = (double)uvw[3 * i], y = (double)uvw[3 * i + 1];
        const double z = (double)uvw[3 * i + 2];
        for (int c = 0; c < num_chan; ++c)
        {
            const double inv_wave = (f0 + df * c) / kC0;
            const double u = x * inv_wave - du;
            const double v = y * inv_wave - dv;
            const double w = z * inv_wave - dw;
            const double phase = kTwoPi * (l * u + m * v + n * w);
            const C2<V> ph{(V)cos(phase), (V)sin(phase)};
            const C2<V> t = cmul2(vis[i * num_chan + c], ph);
            acc.re += t.re;
            acc.im += t.im;
        }
    }
    const int64_t il = s / image_size, im = s - il * image_size;
    const double tv = taper ? taper[il] * taper[im] : 1.0;
    const C2<V> tt = cmul2(acc, C2<V>{(V)tv, V(0)});
    image[s].re += tt.re;
    image[s].im += tt.im;
}

template<typename A, typename B>
__global__ void k_residual(const A* __restrict__ a, const B* __restrict__ b,
        A* __restrict__ out, int64_t n)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) out[i] = a[i] - (A)b[i];
}

// Non-zero pixels of rows x cols (complex: either part non-zero).
template<typename T>
__global__ void k_count_nonzero(const T* __restrict__ img, int64_t rows,
        int64_t cols, int64_t row_stride, int cplx,
        unsigned long long* __restrict__ count)
{
    __shared__ unsigned int part;
    if (threadIdx.x == 0) part = 0;
    __syncthreads();
    unsigned int mine = 0;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
            k < rows * cols; k += (int64_t)gridDim.x * blockDim.x)
    {
        const int64_t r = k / cols, c = k - r * cols;
        const T* p = img + (r * row_stride + c) * (cplx ? 2 : 1);
        if (p[0] != T(0) || (cplx && p[1] != T(0))) ++mine;
    }
    atomicAdd(&part, mine);
    __syncthreads();
    if (threadIdx.x == 0 && part) atomicAdd(count, (unsigned long long)part);
}

bool need_gpu(sdp_Error* status)
{
    if (*status) return false;
    if (sdp_hip::device_available()) return true;
    *status = SDP_ERR_MEM_LOCATION;
    SDP_LOG_ERROR("No GPU available for the gridder utilities.");
    return false;
}

unsigned blocks_of(int64_t n, int t = 256)
{
    return (unsigned)((n + t - 1) / t);
}

const int* int_ptr(const Staged& s)
{
    return s.dev ? (const int*)sdp_mem_data(s.dev) : nullptr;
}

// Shapes the DFT kernels index without bounds checks: lmn [n >= min_dirs,
// 3] of the direction type, channel ranges int32 with one entry per uvw row
// (checked when both are given). Returns false (status set) otherwise.
bool check_dft_shapes(const sdp_Mem* uvws, const sdp_Mem* start_chs,
        const sdp_Mem* end_chs, const sdp_Mem* lmn, int64_t min_dirs,
        sdp_Error* status)
{
    const int64_t rows = sdp_mem_shape_dim(uvws, 0);
    bool ok = sdp_mem_num_dims(lmn) == 2 && sdp_mem_shape_dim(lmn, 1) == 3 &&
            sdp_mem_shape_dim(lmn, 0) >= min_dirs;
    // As the reference, the ranges are used only when both are given.
    const bool ranges = start_chs && end_chs;
    for (const sdp_Mem* c : {start_chs, end_chs})
    {
        if (!ranges) break;
        if (sdp_mem_type(c) != SDP_MEM_INT || sdp_mem_num_elements(c) < rows ||
                !sdp_mem_is_c_contiguous(c))
            ok = false;
    }
    if (!ok)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("lmn must be [n, 3]; start_chs / end_chs int32 arrays "
                "with one entry per uvw row");
    }
    return ok;
}

// Subgrid offsets scaled as sdp_gridder_utils.cpp:171-178.
void offsets(int ou, int ov, int ow, double theta, double w_step,
        double* du, double* dv, double* dw)
{
    *du = *dv = *dw = 0.0;
    if (theta > 0)
    {
        *du = (double)ou / theta;
        *dv = (double)ov / theta;
        *dw = (double)ow * w_step;
    }
}

template<typename IMG, typename DIR>
void image_to_flmn_t(const IMG* image, int size_l, int size_m, double theta,
        double shear_u, double shear_v, const double* taper, double* flux,
        DIR* lmn)
{
    int64_t k = 0;
    for (int il = 0; il < size_l; ++il)
    {
        const double l = (il - size_l / 2) * theta / size_l;
        for (int im = 0; im < size_m; ++im)
        {
            const double m = (im - size_m / 2) * theta / size_m;
            if (flux)
            {
                const IMG v = image[(int64_t)il * size_m + im];
                if (v == IMG(0)) continue;
                const double tv = taper ? taper[il] * taper[im] : 1.0;
                flux[k] = std::real(v) * tv;
            }
            lmn[3 * k] = (DIR)l;
            lmn[3 * k + 1] = (DIR)m;
            lmn[3 * k + 2] = (DIR)lm_to_n(l, m, shear_u, shear_v);
            ++k;
        }
    }
}

// Non-zero pixels over the whole size_l x size_m region the fill loop of
// image_to_flmn_t visits (the exported count follows the reference and
// sees only shape[0] columns, so it cannot size the outputs of a
// non-square image).
template<typename IMG>
int64_t count_nonzero_host(const IMG* image, int size_l, int size_m)
{
    int64_t k = 0;
    for (int64_t i = 0; i < (int64_t)size_l * size_m; ++i)
        k += image[i] != IMG(0);
    return k;
}

} // namespace

extern "C" {

int64_t sdp_gridder_count_nonzero_pixels(const sdp_Mem* image,
        sdp_Error* status)
{
    if (*status) return 0;
    const sdp_MemType t = sdp_mem_type(image);
    const int kind = any_kind(t);
    if (kind < 0)
    {
        *status = SDP_ERR_DATA_TYPE;
        return 0;
    }
    if (sdp_mem_num_dims(image) != 2 || !sdp_mem_is_c_contiguous(image))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Image must be a 2-D C-contiguous array");
        return 0;
    }
    if (!need_gpu(status)) return 0;
    Staged im;
    im.init(image, status);
    if (*status) return 0;
    // sdp_gridder_utils.cpp:106-123: image_size = shape[0] in both axes.
    const int64_t n0 = sdp_mem_shape_dim(image, 0);
    const int64_t n1 = sdp_mem_shape_dim(image, 1);
    const int64_t cols = n0 < n1 ? n0 : n1;
    unsigned long long* d_count = nullptr;
    SDP_HIP_CHECK(hipMalloc((void**)&d_count, sizeof(*d_count)), status);
    if (*status) return 0;
    SDP_HIP_CHECK(hipMemset(d_count, 0, sizeof(*d_count)), status);
    const unsigned blocks = (unsigned)std::min<int64_t>(4096,
            std::max<int64_t>(1, blocks_of(n0 * cols)));
    const int cplx = kind >= 2;
    if (kind == 0 || kind == 2)
        k_count_nonzero<float><<<blocks, 256>>>(
                (const float*)sdp_mem_data(im.dev), n0, cols, n1, cplx,
                d_count);
    else
        k_count_nonzero<double><<<blocks, 256>>>(
                (const double*)sdp_mem_data(im.dev), n0, cols, n1, cplx,
                d_count);
    SDP_HIP_CHECK_LAUNCH(status);
    unsigned long long h = 0;
    SDP_HIP_CHECK(hipMemcpy(&h, d_count, sizeof(h), hipMemcpyDeviceToHost),
            status);
    (void)hipFree(d_count);
    return (int64_t)h;
}

void sdp_gridder_dft(const sdp_Mem* uvws, const sdp_Mem* start_chs,
        const sdp_Mem* end_chs, const sdp_Mem* flux, const sdp_Mem* lmn,
        int subgrid_offset_u, int subgrid_offset_v, int subgrid_offset_w,
        double theta, double w_step, double freq0_hz, double dfreq_hz,
        sdp_Mem* vis, sdp_Error* status)
{
    if (*status) return;
    const sdp_MemType dir_t = sdp_mem_type(lmn), uvw_t = sdp_mem_type(uvws);
    const sdp_MemType vis_t = sdp_mem_type(vis);
    // sdp_gridder_utils.cpp:1056-1090: (double lmn, double uvw, complex
    // double vis) and the float triple; fluxes are double.
    const bool dbl = dir_t == SDP_MEM_DOUBLE && uvw_t == SDP_MEM_DOUBLE &&
            vis_t == SDP_MEM_COMPLEX_DOUBLE;
    const bool flt = dir_t == SDP_MEM_FLOAT && uvw_t == SDP_MEM_FLOAT &&
            vis_t == SDP_MEM_COMPLEX_FLOAT;
    if ((!dbl && !flt) || sdp_mem_type(flux) != SDP_MEM_DOUBLE)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data types");
        return;
    }
    if (sdp_mem_num_dims(vis) != 2 || sdp_mem_num_dims(uvws) != 2 ||
            sdp_mem_shape_dim(uvws, 0) != sdp_mem_shape_dim(vis, 0) ||
            sdp_mem_shape_dim(uvws, 1) != 3 ||
            sdp_mem_shape_dim(lmn, 0) != sdp_mem_shape_dim(flux, 0) ||
            !sdp_mem_is_c_contiguous(vis) || !sdp_mem_is_c_contiguous(uvws) ||
            !sdp_mem_is_c_contiguous(lmn) || !sdp_mem_is_c_contiguous(flux))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Inconsistent array shapes");
        return;
    }
    if (!check_dft_shapes(uvws, start_chs, end_chs, lmn,
            sdp_mem_shape_dim(flux, 0), status))
        return;
    if (!need_gpu(status)) return;
    Staged u, s, e, f, d, v;
    u.init(uvws, status);
    if (start_chs && end_chs)
    {
        s.init(start_chs, status);
        e.init(end_chs, status);
    }
    f.init(flux, status);
    d.init(lmn, status);
    v.init(vis, status);
    if (*status) return;
    double du, dv, dw;
    offsets(subgrid_offset_u, subgrid_offset_v, subgrid_offset_w, theta,
            w_step, &du, &dv, &dw);
    const int64_t rows = sdp_mem_shape_dim(vis, 0);
    const int nchan = (int)sdp_mem_shape_dim(vis, 1);
    const int nsrc = (int)sdp_mem_shape_dim(flux, 0);
    const int64_t n = rows * nchan;
    if (n > 0)
    {
        if (dbl)
            k_dft<double, double, double><<<blocks_of(n), 256>>>(
                    (const double*)sdp_mem_data(u.dev), int_ptr(s),
                    int_ptr(e), (const double*)sdp_mem_data(f.dev),
                    (const double*)sdp_mem_data(d.dev), nsrc, du, dv, dw,
                    freq0_hz, dfreq_hz, rows, nchan,
                    (C2<double>*)sdp_mem_data(v.dev));
        else
            k_dft<float, float, float><<<blocks_of(n), 256>>>(
                    (const float*)sdp_mem_data(u.dev), int_ptr(s),
                    int_ptr(e), (const double*)sdp_mem_data(f.dev),
                    (const float*)sdp_mem_data(d.dev), nsrc, du, dv, dw,
                    freq0_hz, dfreq_hz, rows, nchan,
                    (C2<float>*)sdp_mem_data(v.dev));
        SDP_HIP_CHECK_LAUNCH(status);
    }
    v.write_back(status);
}

void sdp_gridder_idft(const sdp_Mem* uvws, const sdp_Mem* vis,
        const sdp_Mem* start_chs, const sdp_Mem* end_chs, const sdp_Mem* lmn,
        const sdp_Mem* image_taper_1d, int subgrid_offset_u,
        int subgrid_offset_v, int subgrid_offset_w, double theta,
        double w_step, double freq0_hz, double dfreq_hz, sdp_Mem* image,
        sdp_Error* status)
{
    if (*status) return;
    const sdp_MemType img_t = sdp_mem_type(image), dir_t = sdp_mem_type(lmn);
    const sdp_MemType uvw_t = sdp_mem_type(uvws), vis_t = sdp_mem_type(vis);
    // sdp_gridder_utils.cpp:1126-1156.
    const bool dbl = dir_t == SDP_MEM_DOUBLE &&
            img_t == SDP_MEM_COMPLEX_DOUBLE && uvw_t == SDP_MEM_DOUBLE &&
            vis_t == SDP_MEM_COMPLEX_DOUBLE;
    const bool flt = dir_t == SDP_MEM_FLOAT &&
            img_t == SDP_MEM_COMPLEX_FLOAT && uvw_t == SDP_MEM_FLOAT &&
            vis_t == SDP_MEM_COMPLEX_FLOAT;
    if (!dbl && !flt)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data types");
        return;
    }
    const int64_t size = sdp_mem_shape_dim(image, 0);
    if (sdp_mem_num_dims(image) != 2 || sdp_mem_shape_dim(image, 1) != size ||
            sdp_mem_num_dims(vis) != 2 || sdp_mem_num_dims(uvws) != 2 ||
            sdp_mem_shape_dim(uvws, 1) != 3 ||
            sdp_mem_shape_dim(lmn, 0) < size * size ||
            sdp_mem_shape_dim(uvws, 0) != sdp_mem_shape_dim(vis, 0) ||
            (image_taper_1d &&
             (sdp_mem_type(image_taper_1d) != SDP_MEM_DOUBLE ||
              sdp_mem_shape_dim(image_taper_1d, 0) < size)) ||
            !sdp_mem_is_c_contiguous(image) || !sdp_mem_is_c_contiguous(vis) ||
            !sdp_mem_is_c_contiguous(uvws) || !sdp_mem_is_c_contiguous(lmn))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Inconsistent array shapes");
        return;
    }
    if (!check_dft_shapes(uvws, start_chs, end_chs, lmn, size * size, status))
        return;
    if (!need_gpu(status)) return;
    Staged u, vv, s, e, d, tp, im;
    u.init(uvws, status);
    vv.init(vis, status);
    if (start_chs && end_chs)
    {
        s.init(start_chs, status);
        e.init(end_chs, status);
    }
    d.init(lmn, status);
    tp.init(image_taper_1d, status);
    im.init(image, status);
    if (*status) return;
    double du, dv, dw;
    offsets(subgrid_offset_u, subgrid_offset_v, subgrid_offset_w, theta,
            w_step, &du, &dv, &dw);
    const int64_t rows = sdp_mem_shape_dim(vis, 0);
    const int nchan = (int)sdp_mem_shape_dim(vis, 1);
    const double* taper = image_taper_1d ?
            (const double*)sdp_mem_data(tp.dev) : nullptr;
    const int64_t n = size * size;
    if (n > 0)
    {
        if (dbl)
            k_idft<double, double, double><<<blocks_of(n), 256>>>(
                    (const double*)sdp_mem_data(u.dev),
                    (const C2<double>*)sdp_mem_data(vv.dev), int_ptr(s),
                    int_ptr(e), (const double*)sdp_mem_data(d.dev), taper,
                    du, dv, dw, freq0_hz, dfreq_hz, rows, nchan, size,
                    (C2<double>*)sdp_mem_data(im.dev));
        else
            k_idft<float, float, float><<<blocks_of(n), 256>>>(
                    (const float*)sdp_mem_data(u.dev),
                    (const C2<float>*)sdp_mem_data(vv.dev), int_ptr(s),
                    int_ptr(e), (const float*)sdp_mem_data(d.dev), taper,
                    du, dv, dw, freq0_hz, dfreq_hz, rows, nchan, size,
                    (C2<float>*)sdp_mem_data(im.dev));
        SDP_HIP_CHECK_LAUNCH(status);
    }
    im.write_back(status);
}

void sdp_gridder_image_to_flmn(const sdp_Mem* image, double theta,
        double shear_u, double shear_v, const sdp_Mem* image_taper_1d,
        sdp_Mem* flux, sdp_Mem* lmn, sdp_Error* status)
{
    if (*status) return;
    const sdp_MemType img_t = sdp_mem_type(image);
    const sdp_MemType flux_t = flux ? sdp_mem_type(flux) : SDP_MEM_DOUBLE;
    const sdp_MemType dir_t = sdp_mem_type(lmn);
    // sdp_gridder_utils.cpp:1255-1300.
    const bool ok = flux_t == SDP_MEM_DOUBLE && (
            (img_t == SDP_MEM_DOUBLE && dir_t == SDP_MEM_DOUBLE) ||
            (img_t == SDP_MEM_FLOAT && dir_t == SDP_MEM_FLOAT) ||
            (img_t == SDP_MEM_COMPLEX_DOUBLE && dir_t == SDP_MEM_DOUBLE) ||
            (img_t == SDP_MEM_COMPLEX_FLOAT && (dir_t == SDP_MEM_FLOAT ||
                    dir_t == SDP_MEM_DOUBLE)));
    if (!ok)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data types");
        return;
    }
    // Outputs are host tables, as in the reference (CPU views).
    if (sdp_mem_location(lmn) != SDP_MEM_CPU ||
            (flux && sdp_mem_location(flux) != SDP_MEM_CPU) ||
            (image_taper_1d && sdp_mem_location(image_taper_1d) != SDP_MEM_CPU))
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("flux, lmn and image_taper_1d must be in CPU memory");
        return;
    }
    const int size_l = (int)sdp_mem_shape_dim(image, 0);
    const int size_m = (int)sdp_mem_shape_dim(image, 1);
    int64_t needed = (int64_t)size_l * size_m;
    sdp_Mem* host_img = nullptr;
    const void* img = nullptr;
    if (flux)
    {
        if (sdp_mem_location(image) != SDP_MEM_CPU)
        {
            host_img = sdp_mem_create_copy(image, SDP_MEM_CPU, status);
            if (*status) return;
            img = sdp_mem_data_const(host_img);
        }
        else
        {
            img = sdp_mem_data_const(image);
        }
        if (sdp_mem_num_dims(image) != 2 || !sdp_mem_is_c_contiguous(image))
        {
            *status = SDP_ERR_INVALID_ARGUMENT;
            SDP_LOG_ERROR("Image must be a 2-D C-contiguous array");
            sdp_mem_free(host_img);
            return;
        }
        if (img_t == SDP_MEM_DOUBLE)
            needed = count_nonzero_host((const double*)img, size_l, size_m);
        else if (img_t == SDP_MEM_FLOAT)
            needed = count_nonzero_host((const float*)img, size_l, size_m);
        else if (img_t == SDP_MEM_COMPLEX_DOUBLE)
            needed = count_nonzero_host((const std::complex<double>*)img,
                    size_l, size_m);
        else
            needed = count_nonzero_host((const std::complex<float>*)img,
                    size_l, size_m);
        if (sdp_mem_shape_dim(flux, 0) < needed)
        {
            *status = SDP_ERR_INVALID_ARGUMENT;
            SDP_LOG_ERROR("flux array too small");
        }
    }
    if (!*status && image_taper_1d &&
            (sdp_mem_type(image_taper_1d) != SDP_MEM_DOUBLE ||
             sdp_mem_num_elements(image_taper_1d) <
                     (int64_t)std::max(size_l, size_m)))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("image_taper_1d must be a double array of at least "
                "max(image dims) entries");
    }
    if (!*status && (sdp_mem_num_dims(lmn) != 2 ||
            sdp_mem_shape_dim(lmn, 0) < needed ||
            sdp_mem_shape_dim(lmn, 1) != 3 || !sdp_mem_is_c_contiguous(lmn)))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("lmn must be a C-contiguous [n, 3] array");
    }
    if (*status)
    {
        sdp_mem_free(host_img);
        return;
    }
    const double* taper = image_taper_1d ?
            (const double*)sdp_mem_data_const(image_taper_1d) : nullptr;
    double* fl = flux ? (double*)sdp_mem_data(flux) : nullptr;
    void* out = sdp_mem_data(lmn);
#define SDP_FLMN(IMG, DIR) image_to_flmn_t<IMG, DIR>((const IMG*)img, \
        size_l, size_m, theta, shear_u, shear_v, taper, fl, (DIR*)out)
    if (img_t == SDP_MEM_DOUBLE) SDP_FLMN(double, double);
    else if (img_t == SDP_MEM_FLOAT) SDP_FLMN(float, float);
    else if (img_t == SDP_MEM_COMPLEX_DOUBLE)
        SDP_FLMN(std::complex<double>, double);
    else if (dir_t == SDP_MEM_FLOAT) SDP_FLMN(std::complex<float>, float);
    else SDP_FLMN(std::complex<float>, double);
#undef SDP_FLMN
    sdp_mem_free(host_img);
}

void sdp_gridder_residual(const sdp_Mem* a, const sdp_Mem* b, sdp_Mem* out,
        sdp_Error* status)
{
    if (*status) return;
    const sdp_MemType ta = sdp_mem_type(a), tb = sdp_mem_type(b);
    if (sdp_mem_num_dims(a) != 2 || sdp_mem_num_dims(b) != 2 ||
            sdp_mem_num_dims(out) != 2)
    {
        SDP_LOG_ERROR("All arrays must be 2D");
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    if (sdp_mem_shape_dim(a, 0) != sdp_mem_shape_dim(b, 0) ||
            sdp_mem_shape_dim(a, 1) != sdp_mem_shape_dim(b, 1) ||
            sdp_mem_shape_dim(a, 0) != sdp_mem_shape_dim(out, 0) ||
            sdp_mem_shape_dim(a, 1) != sdp_mem_shape_dim(out, 1))
    {
        SDP_LOG_ERROR("All arrays must have the same shape");
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    if (ta != sdp_mem_type(out))
    {
        SDP_LOG_ERROR("Arrays 'a' and 'out' must be of the same type");
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    // sdp_gridder_utils.cpp:1418-1423.
    if (sdp_mem_location(out) != SDP_MEM_CPU)
    {
        SDP_LOG_ERROR("Output residual must be in CPU memory");
        *status = SDP_ERR_MEM_LOCATION;
        return;
    }
    const bool ok = (ta == tb && any_kind(ta) >= 0) ||
            (ta == SDP_MEM_COMPLEX_DOUBLE && tb == SDP_MEM_COMPLEX_FLOAT) ||
            (ta == SDP_MEM_DOUBLE && tb == SDP_MEM_FLOAT);
    if (!ok)
    {
        SDP_LOG_ERROR("Unsupported data types for residual calculation");
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (!sdp_mem_is_c_contiguous(a) || !sdp_mem_is_c_contiguous(b) ||
            !sdp_mem_is_c_contiguous(out))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    if (!need_gpu(status)) return;
    Staged da, db, dout;
    da.init(a, status);
    db.init(b, status);
    dout.init(out, status);
    if (*status) return;
    const int64_t n = sdp_mem_num_elements(a) *
            (sdp_mem_is_complex(a) ? 2 : 1);
    const bool a_dbl = ta == SDP_MEM_DOUBLE || ta == SDP_MEM_COMPLEX_DOUBLE;
    const bool b_dbl = tb == SDP_MEM_DOUBLE || tb == SDP_MEM_COMPLEX_DOUBLE;
    if (n > 0)
    {
        void* po = sdp_mem_data(dout.dev);
        const void* pa = sdp_mem_data(da.dev);
        const void* pb = sdp_mem_data(db.dev);
        if (a_dbl && b_dbl)
            k_residual<double, double><<<blocks_of(n), 256>>>(
                    (const double*)pa, (const double*)pb, (double*)po, n);
        else if (a_dbl)
            k_residual<double, float><<<blocks_of(n), 256>>>(
                    (const double*)pa, (const float*)pb, (double*)po, n);
        else
            k_residual<float, float><<<blocks_of(n), 256>>>(
                    (const float*)pa, (const float*)pb, (float*)po, n);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    dout.write_back(status);
}

} // extern "C"
