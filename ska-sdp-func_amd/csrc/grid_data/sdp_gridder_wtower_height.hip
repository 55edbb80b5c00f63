// W-tower height search (sdp_gridder_wtower_height.cpp of ska-sdp-func
// 1.2.2, :16-316): degrid a worst-case image at growing w with the GPU
// w-towers gridder and compare with the direct Fourier sum.
#include <algorithm>
#include <cmath>
#include <vector>

#include "ska-sdp-func/grid_data/sdp_gridder_utils.h"
#include "ska-sdp-func/grid_data/sdp_gridder_wtower_height.h"
#include "ska-sdp-func/grid_data/sdp_gridder_wtower_uvw.h"
#include "wtower_math.h"
#include "wtower_ops.h"
#include "../fft/fft2d.h"
#include "../utility/sdp_hip.h"

using namespace sdp_wt;

namespace {

__global__ void k_scale_c128(double* data, int64_t n, double factor)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < 2 * n) data[i] *= factor;
}

// Pixel positions of sdp_gridder_worst_case_image (.cpp:288-315), with
// their values; fov_edge as the reference computes it.
struct Source
{
    int il, im;
    double flux;
};

bool worst_case_sources(int image_size, double theta, double fov,
        std::vector<Source>* src)
{
    int fov_edge = int(image_size / theta * fov / 2);
    while (fov_edge != 0 && image_size % fov_edge == 0) fov_edge -= 1;
    if (fov_edge == 0) return false;
    const int c = image_size / 2;
    src->clear();
    src->push_back({c + fov_edge, c + fov_edge, 0.3});
    src->push_back({c - fov_edge, c - fov_edge, 0.2});
    src->push_back({c + fov_edge, c - fov_edge - 1, 0.3});
    src->push_back({c - fov_edge - 1, c + fov_edge, 0.2});
    return true;
}

sdp_Mem* gpu_array(sdp_MemType type, int ndim, const int64_t* shape,
        sdp_Error* status)
{
    sdp_Mem* m = sdp_mem_create(type, SDP_MEM_GPU, ndim, shape, status);
    sdp_mem_clear_contents(m, status);
    return m;
}

// find_gridder_accuracy (.cpp:16-184).
double gridder_accuracy(sdp_GridderWtowerUVW* kernel, double fov,
        double subgrid_frac, int num_samples, double w, sdp_Error* status)
{
    if (*status) return 0;
    const int image_size = sdp_gridder_wtower_uvw_image_size(kernel);
    const int subgrid_size = sdp_gridder_wtower_uvw_subgrid_size(kernel);
    const double theta = sdp_gridder_wtower_uvw_theta(kernel);
    const double shear_u = sdp_gridder_wtower_uvw_shear_u(kernel);
    const double shear_v = sdp_gridder_wtower_uvw_shear_v(kernel);
    if (num_samples == 0) num_samples = 3;
    const int64_t num_rows = (int64_t)num_samples * num_samples;

    std::vector<Source> src;
    if (!worst_case_sources(image_size, theta, fov, &src))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Field of view too small for the image size");
        return 0;
    }
    // image_to_flmn visits non-zero pixels in row-major order.
    std::sort(src.begin(), src.end(), [](const Source& a, const Source& b) {
        return a.il != b.il ? a.il < b.il : a.im < b.im;
    });

    const int64_t image_shape[] = {image_size, image_size};
    const int64_t sub_shape[] = {subgrid_size, subgrid_size};
    const int64_t uvw_shape[] = {num_rows, 3};
    const int64_t vis_shape[] = {num_rows, 1};
    sdp_Mem* image = gpu_array(SDP_MEM_COMPLEX_DOUBLE, 2, image_shape,
            status);
    sdp_Mem* subgrid = gpu_array(SDP_MEM_COMPLEX_DOUBLE, 2, sub_shape,
            status);
    if (*status)
    {
        sdp_mem_free(image);
        sdp_mem_free(subgrid);
        return 0;
    }
    for (const Source& s : src)
    {
        const double v[2] = {s.flux, 0.0};
        SDP_HIP_CHECK(hipMemcpy((double*)sdp_mem_data(image) +
                2 * ((int64_t)s.il * image_size + s.im), v, sizeof(v),
                hipMemcpyHostToDevice), status);
    }
    sdp_gridder_wtower_uvw_degrid_correct(kernel, image, 0, 0, 0, status);
    sdp_fft::Plan2D* fft_grid = sdp_fft::create_2d(image_size, image_size,
            true, status);
    sdp_fft::Plan2D* ifft_sub = sdp_fft::create_2d(subgrid_size,
            subgrid_size, true, status);
    double* d_img = (double*)sdp_mem_data(image);
    double* d_sub = (double*)sdp_mem_data(subgrid);
    wt_fft_phase<double>(d_img, image_size, image_size, status);
    if (!*status) sdp_fft::exec_2d(fft_grid, d_img, true, 0, status);
    wt_fft_phase<double>(d_img, image_size, image_size, status);
    sdp_gridder_subgrid_cut_out(image, 0, 0, subgrid, status);
    wt_fft_phase<double>(d_sub, subgrid_size, subgrid_size, status);
    if (!*status) sdp_fft::exec_2d(ifft_sub, d_sub, false, 0, status);
    wt_fft_phase<double>(d_sub, subgrid_size, subgrid_size, status);
    const int64_t n_sub = (int64_t)subgrid_size * subgrid_size;
    k_scale_c128<<<(unsigned)((2 * n_sub + 255) / 256), 256>>>(d_sub, n_sub,
            1.0 / n_sub);
    SDP_HIP_CHECK_LAUNCH(status);
    sdp_fft::destroy_2d(fft_grid);
    sdp_fft::destroy_2d(ifft_sub);
    sdp_mem_free(image);

    // Sample points (.cpp:120-134).
    if (subgrid_frac == 0.0) subgrid_frac = 2.0 / 3.0;
    const double start = -subgrid_size * subgrid_frac / theta / 2;
    const double end = subgrid_size * subgrid_frac / theta / 2;
    const double step = (end - start) / (num_samples - 1);
    std::vector<double> uvw(3 * num_rows);
    for (int i = 0, index = 0; i < num_samples; ++i)
        for (int j = 0; j < num_samples; ++j, ++index)
        {
            uvw[3 * index + 0] = start + j * step;
            uvw[3 * index + 1] = start + i * step;
            uvw[3 * index + 2] = w;
        }
    std::vector<int> ones(num_rows, 1);
    sdp_Mem* d_uvw = gpu_array(SDP_MEM_DOUBLE, 2, uvw_shape, status);
    sdp_Mem* d_start = gpu_array(SDP_MEM_INT, 1, &num_rows, status);
    sdp_Mem* d_end = gpu_array(SDP_MEM_INT, 1, &num_rows, status);
    sdp_Mem* d_vis = gpu_array(SDP_MEM_COMPLEX_DOUBLE, 2, vis_shape, status);
    if (!*status)
    {
        SDP_HIP_CHECK(hipMemcpy(sdp_mem_data(d_uvw), uvw.data(),
                uvw.size() * sizeof(double), hipMemcpyHostToDevice), status);
        SDP_HIP_CHECK(hipMemcpy(sdp_mem_data(d_end), ones.data(),
                ones.size() * sizeof(int), hipMemcpyHostToDevice), status);
    }
    sdp_gridder_wtower_uvw_degrid(kernel, subgrid, 0, 0, 0, kC0, kC0, d_uvw,
            d_start, d_end, d_vis, -1, -1, status);
    std::vector<double> vis_test(2 * num_rows, 0.0);
    if (!*status)
        SDP_HIP_CHECK(hipMemcpy(vis_test.data(), sdp_mem_data(d_vis),
                vis_test.size() * sizeof(double), hipMemcpyDeviceToHost),
                status);
    sdp_mem_free(subgrid);
    sdp_mem_free(d_uvw);
    sdp_mem_free(d_start);
    sdp_mem_free(d_end);
    sdp_mem_free(d_vis);
    if (*status) return 0;

    // Direct Fourier sum (.cpp:150-176), then rms (rms_diff).
    double sum_sq = 0.0;
    for (int64_t r = 0; r < num_rows; ++r)
    {
        double re = 0.0, im = 0.0;
        for (const Source& s : src)
        {
            const double l = (s.il - image_size / 2) * theta / image_size;
            const double m = (s.im - image_size / 2) * theta / image_size;
            const double n = lm_to_n(l, m, shear_u, shear_v);
            const double phase = -2.0 * M_PI * (uvw[3 * r] * l +
                    uvw[3 * r + 1] * m + uvw[3 * r + 2] * n);
            re += s.flux * cos(phase);
            im += s.flux * sin(phase);
        }
        const double dr = vis_test[2 * r] - re;
        const double di = vis_test[2 * r + 1] - im;
        sum_sq += dr * dr + di * di;
    }
    return sqrt(sum_sq / num_rows);
}

} // namespace

extern "C" {

double sdp_gridder_determine_max_w_tower_height(int image_size,
        int subgrid_size, double theta, double w_step, double shear_u,
        double shear_v, int support, int oversampling, int w_support,
        int w_oversampling, double fov, double subgrid_frac, int num_samples,
        double target_err, sdp_Error* status)
{
    if (*status) return 0.0;
    sdp_GridderWtowerUVW* kernel = sdp_gridder_wtower_uvw_create(image_size,
            subgrid_size, theta, w_step, shear_u, shear_v, support,
            oversampling, w_support, w_oversampling, status);
    if (*status)
    {
        sdp_gridder_wtower_uvw_free(kernel);
        return 0.0;
    }
    if (target_err == 0.0)
        target_err = 2 * gridder_accuracy(kernel, fov, subgrid_frac,
                num_samples, 0.0, status);
    // Exponential then binary search on the height (.cpp:226-265).
    double result = 0.0;
    int iw = 1, diw = 1;
    bool accelerate = true;
    while (!*status)
    {
        const double err = gridder_accuracy(kernel, fov, subgrid_frac,
                num_samples, iw * w_step, status);
        if (err < target_err)
        {
            if (accelerate)
                diw *= 2;
            else if (diw > 1)
                diw /= 2;
            else
            {
                result = 2 * iw;
                break;
            }
            iw += diw;
        }
        else if (diw > 1)
        {
            diw /= 2;
            iw -= diw;
            accelerate = false;
        }
        else
        {
            result = 2 * (iw - 1);
            break;
        }
    }
    sdp_gridder_wtower_uvw_free(kernel);
    return result;
}

void sdp_gridder_worst_case_image(double theta, double fov, sdp_Mem* image,
        sdp_Error* status)
{
    if (*status) return;
    const int image_size = (int)sdp_mem_shape_dim(image, 0);
    if (sdp_mem_num_dims(image) != 2 ||
            image_size != sdp_mem_shape_dim(image, 1))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Image must be square");
        return;
    }
    if (sdp_mem_type(image) != SDP_MEM_COMPLEX_DOUBLE)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data type");
        return;
    }
    if (sdp_mem_location(image) != SDP_MEM_CPU)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Image must be in CPU memory");
        return;
    }
    std::vector<Source> src;
    if (!worst_case_sources(image_size, theta, fov, &src))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Field of view too small for the image size");
        return;
    }
    sdp_mem_clear_contents(image, status);
    double* p = (double*)sdp_mem_data(image);
    for (const Source& s : src)
        p[2 * ((int64_t)s.il * image_size + s.im)] = s.flux;
}

} // extern "C"
