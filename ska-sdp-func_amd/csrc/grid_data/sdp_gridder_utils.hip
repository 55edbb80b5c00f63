// Gridder utilities of the w-towers path: element-wise sub-grid kernels and
// the drop-in C ABI of include/ska-sdp-func/grid_data/sdp_gridder_utils.h.
//
// Replaces the subset of src/ska-sdp-func/grid_data/sdp_gridder_utils.cpp/.cu
// and sdp_gridder_clamp_channels.cpp/.cu (ska-sdp-func 1.2.2) used by the
// w-towers gridder. Array operations run on the GPU; CPU arrays are staged
// through device memory. The table generators fill CPU arrays (as the
// reference); rms_diff reduces on the host after copying (as the reference).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "ska-sdp-func/grid_data/sdp_gridder_clamp_channels.h"
#include "ska-sdp-func/grid_data/sdp_gridder_utils.h"
#include "wtower_math.h"
#include "wtower_ops.h"
#include "../utility/sdp_hip.h"

namespace sdp_wt {

namespace {

__global__ void k_scale_inv(AnyView out, AnyView in1,
        const Cx<double>* __restrict__ w_pattern, int exponent, int64_t n)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Cx<double> w = (exponent == 1) ? w_pattern[i] :
            cpow_int(w_pattern[i], exponent);
    out.store(i, cdiv(in1.load(i), w));
}

__global__ void k_accum(AnyView out, AnyView in1,
        const Cx<double>* __restrict__ w_pattern, int exponent, int64_t n)
{
#pragma clang fp contract(off)
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Cx<double> v = in1.load(i);
    Cx<double> o = out.load(i);
    if (out.kind <= 1)
    {
        o.re += v.re;
        out.store(i, o);
        return;
    }
    if (w_pattern && exponent != 0)
    {
        const Cx<double> w = (exponent == 1) ? w_pattern[i] :
                cpow_int(w_pattern[i], exponent);
        v = cmul(v, w);
    }
    o.re += v.re;
    o.im += v.im;
    out.store(i, o);
}

template<typename T>
__global__ void k_fft_phase(T* data, int nx, int ny)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (j >= ny || ((i + j) & 1) == 0) return;
    const int64_t k = 2 * ((int64_t)i * ny + j);
    data[k] = -data[k];
    data[k + 1] = -data[k + 1];
}

__global__ void k_shift_subgrids(char* data, int64_t layer_bytes, int layers)
{
    // subgrids[:-1] = subgrids[1:], in 16-byte words, layer by layer.
    const int64_t words = layer_bytes / 16;
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= words) return;
    uint4* p = (uint4*)data;
    for (int l = 0; l < layers - 1; ++l)
        p[l * words + t] = p[(l + 1) * words + t];
}

template<typename G>
__global__ void k_subgrid_add(G* grid, int64_t gu, int64_t gv,
        const G* sub, int64_t su, int64_t sv, int off_u, int off_v,
        double factor, int complex_)
{
#pragma clang fp contract(off)
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t i = blockIdx.y;
    if (j >= sv) return;
    int64_t i1 = (i + gu / 2 - su / 2 - off_u) % gu;
    int64_t j1 = (j + gv / 2 - sv / 2 - off_v) % gv;
    if (i1 < 0) i1 += gu;
    if (j1 < 0) j1 += gv;
    const G f = (G)factor;
    const int c = complex_ ? 2 : 1;
    for (int k = 0; k < c; ++k)
        grid[c * (i1 * gv + j1) + k] += sub[c * (i * sv + j) + k] * f;
}

template<typename G>
__global__ void k_subgrid_cut_out(const G* grid, int64_t gu, int64_t gv,
        G* sub, int64_t su, int64_t sv, int off_u, int off_v, int complex_)
{
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t i = blockIdx.y;
    if (j >= sv) return;
    int64_t i1 = (i + gu / 2 - su / 2 + off_u) % gu;
    int64_t j1 = (j + gv / 2 - sv / 2 + off_v) % gv;
    if (i1 < 0) i1 += gu;
    if (j1 < 0) j1 += gv;
    const int c = complex_ ? 2 : 1;
    for (int k = 0; k < c; ++k)
        sub[c * (i * sv + j) + k] = grid[c * (i1 * gv + j1) + k];
}

__global__ void k_sum_diff(const int* a, const int* b, int64_t s, int64_t e,
        unsigned long long* out)
{
    __shared__ long long part[256];
    long long acc = 0;
    for (int64_t i = s + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
            i < e; i += (int64_t)gridDim.x * blockDim.x)
        acc += (long long)a[i] - b[i];
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1)
    {
        if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0)
        atomicAdd(out, (unsigned long long)part[0]);
}

// Per-block partial bounds of the three scaled coordinates
// (sdp_gridder_utils.cpp:682-719; starts at +/-inf).
template<typename U>
__global__ void k_uvw_bounds(const U* __restrict__ uvws, int64_t rows,
        double f0, double df, const int* __restrict__ start_chs,
        const int* __restrict__ end_chs, double* __restrict__ part)
{
#pragma clang fp contract(off)
    __shared__ double s_lo[3][256], s_hi[3][256];
    double lo[3] = {INFINITY, INFINITY, INFINITY};
    double hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
            i < rows; i += (int64_t)gridDim.x * blockDim.x)
    {
        const int s = start_chs[i], e = end_chs[i];
        if (s >= e) continue;
        for (int j = 0; j < 3; ++j)
        {
            const double u = (double)uvws[3 * i + j];
            const double u0 = f0 * u / kC0;
            const double du = df * u / kC0;
            if (u >= 0)
            {
                lo[j] = fmin(u0 + s * du, lo[j]);
                hi[j] = fmax(u0 + (e - 1) * du, hi[j]);
            }
            else
            {
                hi[j] = fmax(u0 + s * du, hi[j]);
                lo[j] = fmin(u0 + (e - 1) * du, lo[j]);
            }
        }
    }
    for (int j = 0; j < 3; ++j)
    {
        s_lo[j][threadIdx.x] = lo[j];
        s_hi[j][threadIdx.x] = hi[j];
    }
    __syncthreads();
    for (int off = blockDim.x / 2; off > 0; off >>= 1)
    {
        if ((int)threadIdx.x < off)
            for (int j = 0; j < 3; ++j)
            {
                s_lo[j][threadIdx.x] = fmin(s_lo[j][threadIdx.x],
                        s_lo[j][threadIdx.x + off]);
                s_hi[j][threadIdx.x] = fmax(s_hi[j][threadIdx.x],
                        s_hi[j][threadIdx.x + off]);
            }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int j = 0; j < 3; ++j)
        {
            part[6 * blockIdx.x + j] = s_lo[j][0];
            part[6 * blockIdx.x + 3 + j] = s_hi[j][0];
        }
}

// sdp_gridder_clamp_channels.cpp:8-62 / 64-150 (uv: dims 0 then 1).
template<typename U>
__global__ void k_clamp(const U* __restrict__ uvws, int dim0, int ndims,
        double f0, double df, const int* __restrict__ s_in,
        const int* __restrict__ e_in, double min0, double max0, double min1,
        double max1, int* __restrict__ s_out, int* __restrict__ e_out,
        int64_t r0, int64_t r1)
{
#pragma clang fp contract(off)
    const int64_t i = r0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= r1) return;
    int s = s_in[i], e = e_in[i];
    for (int d = 0; d < ndims; ++d)
    {
        const double x = (double)uvws[3 * i + dim0 + d];
        const double lo = d ? min1 : min0, hi = d ? max1 : max0;
        const double x0 = x * (f0 / kC0);
        const double dx = x * (df / kC0);
        const double eta = fmax(fabs(lo - x0), fabs(hi - x0)) / 2147483645.0;
        if (fabs(dx) > eta)
        {
            const int mins = (int)(int64_t)ceil((lo - x0) / dx);
            const int maxs = (int)(int64_t)ceil((hi - x0) / dx);
            const bool pos = dx > 0;
            s = max(s, pos ? mins : maxs);
            e = min(e, pos ? maxs : mins);
        }
        else if (lo > x0 || hi <= x0)
        {
            s = 0;
            e = 0;
        }
        e = max(e, s);
        if (s >= e) break;
    }
    s_out[i] = s;
    e_out[i] = e;
}

unsigned blocks_of(int64_t n, int t = 256)
{
    return (unsigned)((n + t - 1) / t);
}

bool need_gpu(sdp_Error* status)
{
    if (*status) return false;
    if (sdp_hip::device_available()) return true;
    *status = SDP_ERR_MEM_LOCATION;
    SDP_LOG_ERROR("No GPU available for the gridder utilities.");
    return false;
}

} // namespace

void wt_scale_inv(AnyView out, AnyView in1, const double* w_pattern,
        int exponent, int64_t n, sdp_Error* status)
{
    if (*status || n <= 0) return;
    k_scale_inv<<<blocks_of(n), 256>>>(out, in1,
            (const Cx<double>*)w_pattern, exponent, n);
    SDP_HIP_CHECK_LAUNCH(status);
}

void wt_accum(AnyView out, AnyView in1, const double* w_pattern,
        int exponent, int64_t n, sdp_Error* status)
{
    if (*status || n <= 0) return;
    k_accum<<<blocks_of(n), 256>>>(out, in1, (const Cx<double>*)w_pattern,
            exponent, n);
    SDP_HIP_CHECK_LAUNCH(status);
}

template<typename T>
void wt_fft_phase(T* data, int nx, int ny, sdp_Error* status)
{
    if (*status) return;
    k_fft_phase<T><<<dim3(blocks_of(ny), nx), 256>>>(data, nx, ny);
    SDP_HIP_CHECK_LAUNCH(status);
}

template void wt_fft_phase<float>(float*, int, int, sdp_Error*);
template void wt_fft_phase<double>(double*, int, int, sdp_Error*);

void Staged::init(const sdp_Mem* m, sdp_Error* status)
{
    src = m;
    if (!m || *status) return;
    if (sdp_mem_location(m) == SDP_MEM_GPU)
    {
        dev = const_cast<sdp_Mem*>(m);
        return;
    }
    dev = sdp_mem_create_copy(m, SDP_MEM_GPU, status);
    copy = true;
}

void Staged::write_back(sdp_Error* status)
{
    if (copy && dev && !*status)
        sdp_mem_copy_contents(const_cast<sdp_Mem*>(src), dev, 0, 0,
                sdp_mem_num_elements(src), status);
}

Staged::~Staged()
{
    if (copy) sdp_mem_free(dev);
}

// Bounds of the selected channels of device arrays (used by the gridder).
template<typename U>
void uvw_bounds_dev(const U* uvws, int64_t rows, double f0, double df,
        const int* s, const int* e, double lo[3], double hi[3],
        sdp_Error* status)
{
    for (int j = 0; j < 3; ++j)
    {
        lo[j] = INFINITY;
        hi[j] = -INFINITY;
    }
    if (*status || rows <= 0) return;
    const int blocks = (int)std::min<int64_t>(1024, blocks_of(rows));
    double* part = nullptr;
    SDP_HIP_CHECK(hipMalloc(&part, blocks * 6 * sizeof(double)), status);
    if (*status) return;
    k_uvw_bounds<U><<<blocks, 256>>>(uvws, rows, f0, df, s, e, part);
    SDP_HIP_CHECK_LAUNCH(status);
    std::vector<double> h(blocks * 6);
    SDP_HIP_CHECK(hipMemcpy(h.data(), part, h.size() * sizeof(double),
            hipMemcpyDeviceToHost), status);
    (void)hipFree(part);
    if (*status) return;
    for (int b = 0; b < blocks; ++b)
        for (int j = 0; j < 3; ++j)
        {
            lo[j] = std::min(lo[j], h[6 * b + j]);
            hi[j] = std::max(hi[j], h[6 * b + 3 + j]);
        }
}

template void uvw_bounds_dev<float>(const float*, int64_t, double, double,
        const int*, const int*, double*, double*, sdp_Error*);
template void uvw_bounds_dev<double>(const double*, int64_t, double, double,
        const int*, const int*, double*, double*, sdp_Error*);

} // namespace sdp_wt

using namespace sdp_wt;

namespace {

bool same_shape_2d(const sdp_Mem* a, const sdp_Mem* b)
{
    return sdp_mem_num_dims(a) == 2 && sdp_mem_num_dims(b) == 2 &&
            sdp_mem_shape_dim(a, 0) == sdp_mem_shape_dim(b, 0) &&
            sdp_mem_shape_dim(a, 1) == sdp_mem_shape_dim(b, 1);
}

bool is_complex_type(sdp_MemType t)
{
    return t == SDP_MEM_COMPLEX_FLOAT || t == SDP_MEM_COMPLEX_DOUBLE;
}

bool is_double_type(sdp_MemType t)
{
    return t == SDP_MEM_DOUBLE || t == SDP_MEM_COMPLEX_DOUBLE;
}

} // namespace

extern "C" {

void sdp_gridder_accumulate_scaled_arrays(sdp_Mem* out, const sdp_Mem* in1,
        const sdp_Mem* in2, int exponent, sdp_Error* status)
{
    if (*status) return;
    if (sdp_mem_location(in1) != sdp_mem_location(out) ||
            (in2 && sdp_mem_location(in2) != sdp_mem_location(out)))
    {
        SDP_LOG_ERROR("All arrays must be in the same memory space");
        *status = SDP_ERR_MEM_LOCATION;
        return;
    }
    const sdp_MemType to = sdp_mem_type(out), t1 = sdp_mem_type(in1);
    const sdp_MemType t2 = in2 ? sdp_mem_type(in2) : SDP_MEM_COMPLEX_DOUBLE;
    if (!in2) exponent = 0;
    const bool ok = any_kind(to) >= 0 && any_kind(t1) >= 0 &&
            t2 == SDP_MEM_COMPLEX_DOUBLE &&
            (is_complex_type(to) || is_complex_type(t1));
    if (!ok)
    {
        SDP_LOG_ERROR("Unsupported image data type");
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (!same_shape_2d(out, in1) || (in2 && !same_shape_2d(out, in2)))
    {
        SDP_LOG_ERROR("Arrays must be 2D with the same shape");
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    if (!need_gpu(status)) return;
    Staged o, a, b;
    o.init(out, status);
    a.init(in1, status);
    b.init(in2, status);
    if (*status) return;
    wt_accum(AnyView{sdp_mem_data(o.dev), any_kind(to)},
            AnyView{sdp_mem_data(a.dev), any_kind(t1)},
            in2 ? (const double*)sdp_mem_data(b.dev) : nullptr, exponent,
            sdp_mem_num_elements(out), status);
    o.write_back(status);
}

double sdp_gridder_determine_w_step(double theta, double fov, double shear_u,
        double shear_v, double x0)
{
    return determine_w_step(theta, fov, shear_u, shear_v, x0);
}

void sdp_gridder_make_kernel(const sdp_Mem* window, sdp_Mem* kernel,
        sdp_Error* status)
{
    if (*status) return;
    const sdp_MemType tw = sdp_mem_type(window), tk = sdp_mem_type(kernel);
    if (tw != tk || (tw != SDP_MEM_DOUBLE && tw != SDP_MEM_FLOAT))
    {
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (sdp_mem_location(window) != SDP_MEM_CPU ||
            sdp_mem_location(kernel) != SDP_MEM_CPU)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Kernel tables are generated in CPU memory");
        return;
    }
    if (sdp_mem_num_dims(window) != 1 || sdp_mem_num_dims(kernel) != 2 ||
            sdp_mem_shape_dim(window, 0) != sdp_mem_shape_dim(kernel, 1))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    const int support = (int)sdp_mem_shape_dim(window, 0);
    const int os = (int)sdp_mem_shape_dim(kernel, 0) - 1;
    std::vector<double> w(support);
    for (int i = 0; i < support; ++i)
        w[i] = (tw == SDP_MEM_DOUBLE) ?
                ((const double*)sdp_mem_data_const(window))[i] :
                ((const float*)sdp_mem_data_const(window))[i];
    // make_kernel computes val / support; the reference rounds val to the
    // output type before scaling (.cpp:423).
    const std::vector<double> k = make_kernel(w, os);
    for (size_t i = 0; i < k.size(); ++i)
    {
        if (tk == SDP_MEM_DOUBLE)
            ((double*)sdp_mem_data(kernel))[i] = k[i];
        else
            ((float*)sdp_mem_data(kernel))[i] = (float)((double)(float)(
                    k[i] * support) * (1.0 / support));
    }
}

void sdp_gridder_make_pswf_kernel(int support, sdp_Mem* kernel,
        sdp_Error* status)
{
    if (*status) return;
    if (sdp_mem_num_dims(kernel) != 2)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    const sdp_MemType tk = sdp_mem_type(kernel);
    if (tk != SDP_MEM_DOUBLE && tk != SDP_MEM_FLOAT)
    {
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (sdp_mem_location(kernel) != SDP_MEM_CPU)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Kernel tables are generated in CPU memory");
        return;
    }
    const int vr = (int)sdp_mem_shape_dim(kernel, 1);
    std::vector<double> pswf = generate_pswf(support * (M_PI / 2), vr, false);
    if (vr % 2 == 0) pswf[0] = 1e-15;
    if (tk == SDP_MEM_FLOAT)
        for (double& v : pswf) v = (double)(float)v;
    const int os = (int)sdp_mem_shape_dim(kernel, 0) - 1;
    const std::vector<double> k = make_kernel(pswf, os);
    for (size_t i = 0; i < k.size(); ++i)
    {
        if (tk == SDP_MEM_DOUBLE)
            ((double*)sdp_mem_data(kernel))[i] = k[i];
        else
            ((float*)sdp_mem_data(kernel))[i] = (float)k[i];
    }
}

void sdp_gridder_make_w_pattern(int subgrid_size, double theta,
        double shear_u, double shear_v, double w_step, sdp_Mem* w_pattern,
        sdp_Error* status)
{
    if (*status) return;
    if (sdp_mem_type(w_pattern) != SDP_MEM_COMPLEX_DOUBLE ||
            sdp_mem_location(w_pattern) != SDP_MEM_CPU ||
            sdp_mem_num_dims(w_pattern) != 2 ||
            sdp_mem_num_elements(w_pattern) <
            (int64_t)subgrid_size * subgrid_size)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("w_pattern must be a complex double CPU array of "
                "shape (subgrid_size, subgrid_size)");
        return;
    }
    const std::vector<std::complex<double> > w = make_w_pattern(subgrid_size,
            theta, shear_u, shear_v, w_step);
    memcpy(sdp_mem_data(w_pattern), w.data(), w.size() * 16);
}

double sdp_gridder_rms_diff(const sdp_Mem* a, const sdp_Mem* b,
        sdp_Error* status)
{
    if (*status) return INFINITY;
    if (sdp_mem_num_dims(a) != 2 || sdp_mem_num_dims(b) != 2)
    {
        SDP_LOG_ERROR("Input arrays must be 2D");
        *status = SDP_ERR_INVALID_ARGUMENT;
        return INFINITY;
    }
    if (!same_shape_2d(a, b))
    {
        SDP_LOG_ERROR("Input arrays must have the same shape");
        *status = SDP_ERR_INVALID_ARGUMENT;
        return INFINITY;
    }
    const sdp_MemType ta = sdp_mem_type(a), tb = sdp_mem_type(b);
    const int ka = any_kind(ta), kb = any_kind(tb);
    // Supported (a, b): same type, or a double-precision a with the
    // single-precision b of the same kind (.cpp:1508-1535).
    const bool ok = ka >= 0 && kb >= 0 &&
            is_complex_type(ta) == is_complex_type(tb) &&
            (ta == tb || (is_double_type(ta) && !is_double_type(tb)));
    if (!ok)
    {
        SDP_LOG_ERROR("Unsupported data types for RMS difference "
                "calculation");
        *status = SDP_ERR_DATA_TYPE;
        return INFINITY;
    }
    sdp_Mem* ha = sdp_mem_create_copy(a, SDP_MEM_CPU, status);
    sdp_Mem* hb = sdp_mem_create_copy(b, SDP_MEM_CPU, status);
    double out = INFINITY;
    if (!*status)
    {
        const int64_t n = sdp_mem_num_elements(a);
        const bool single = !is_double_type(ta);
        double sum = 0.0;
        for (int64_t i = 0; i < n; ++i)
        {
            double re = 0, im = 0;
            const void* pa = sdp_mem_data(ha);
            const void* pb = sdp_mem_data(hb);
            auto get = [](const void* p, int kind, int64_t i, double* r,
                    double* m) {
                switch (kind)
                {
                case 0: *r = ((const float*)p)[i]; *m = 0; break;
                case 1: *r = ((const double*)p)[i]; *m = 0; break;
                case 2:
                    *r = ((const float*)p)[2 * i];
                    *m = ((const float*)p)[2 * i + 1];
                    break;
                default:
                    *r = ((const double*)p)[2 * i];
                    *m = ((const double*)p)[2 * i + 1];
                }
            };
            double ar, ai, br, bi;
            get(pa, ka, i, &ar, &ai);
            get(pb, kb, i, &br, &bi);
            if (single)
            {
                re = (float)((float)ar - (float)br);
                im = (float)((float)ai - (float)bi);
                sum += (double)(float)((float)re * (float)re +
                        (float)im * (float)im);
            }
            else
            {
                re = ar - br;
                im = ai - bi;
                sum += re * re + im * im;
            }
        }
        out = std::sqrt(sum / (double)n);
    }
    sdp_mem_free(ha);
    sdp_mem_free(hb);
    return out;
}

void sdp_gridder_scale_inv_array(sdp_Mem* out, const sdp_Mem* in1,
        const sdp_Mem* in2, int exponent, sdp_Error* status)
{
    if (*status) return;
    if (sdp_mem_location(in1) != sdp_mem_location(out) ||
            sdp_mem_location(in2) != sdp_mem_location(out))
    {
        SDP_LOG_ERROR("All arrays must be in the same memory space");
        *status = SDP_ERR_MEM_LOCATION;
        return;
    }
    const sdp_MemType to = sdp_mem_type(out), t1 = sdp_mem_type(in1);
    const bool ok = sdp_mem_type(in2) == SDP_MEM_COMPLEX_DOUBLE &&
            ((to == SDP_MEM_COMPLEX_DOUBLE &&
            (t1 == SDP_MEM_DOUBLE || t1 == SDP_MEM_COMPLEX_DOUBLE)) ||
            (to == SDP_MEM_COMPLEX_FLOAT &&
            (t1 == SDP_MEM_FLOAT || t1 == SDP_MEM_COMPLEX_FLOAT)));
    if (!ok)
    {
        SDP_LOG_ERROR("Unsupported image data type");
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (!same_shape_2d(out, in1) || !same_shape_2d(out, in2))
    {
        SDP_LOG_ERROR("Arrays must be 2D with the same shape");
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    if (!need_gpu(status)) return;
    Staged o, a, b;
    o.init(out, status);
    a.init(in1, status);
    b.init(in2, status);
    if (*status) return;
    wt_scale_inv(AnyView{sdp_mem_data(o.dev), any_kind(to)},
            AnyView{sdp_mem_data(a.dev), any_kind(t1)},
            (const double*)sdp_mem_data(b.dev), exponent,
            sdp_mem_num_elements(out), status);
    o.write_back(status);
}

void sdp_gridder_shift_subgrids(sdp_Mem* subgrids, sdp_Error* status)
{
    if (*status) return;
    const sdp_MemType t = sdp_mem_type(subgrids);
    if (!is_complex_type(t))
    {
        SDP_LOG_ERROR("Unsupported sub-grid data type");
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (sdp_mem_num_dims(subgrids) != 3)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    if (!need_gpu(status)) return;
    Staged s;
    s.init(subgrids, status);
    if (*status) return;
    const int layers = (int)sdp_mem_shape_dim(subgrids, 0);
    const int64_t layer_bytes = sdp_mem_shape_dim(subgrids, 1) *
            sdp_mem_shape_dim(subgrids, 2) * sdp_mem_type_size(t);
    char* base = (char*)sdp_mem_data(s.dev);
    if (layer_bytes % 16 == 0)
    {
        k_shift_subgrids<<<blocks_of(layer_bytes / 16), 256>>>(base,
                layer_bytes, layers);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    else
    {
        for (int l = 0; l + 1 < layers; ++l)
            SDP_HIP_CHECK(hipMemcpyAsync(base + l * layer_bytes,
                    base + (l + 1) * layer_bytes, layer_bytes,
                    hipMemcpyDeviceToDevice, 0), status);
    }
    s.write_back(status);
}

void sdp_gridder_subgrid_add(sdp_Mem* grid, int offset_u, int offset_v,
        const sdp_Mem* subgrid, double factor, sdp_Error* status)
{
    if (*status) return;
    const sdp_MemType tg = sdp_mem_type(grid);
    if (tg != sdp_mem_type(subgrid) || any_kind(tg) < 0)
    {
        SDP_LOG_ERROR("Unsupported grid or sub-grid data type");
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (sdp_mem_location(grid) != sdp_mem_location(subgrid))
    {
        SDP_LOG_ERROR("All arrays must be in the same memory space");
        *status = SDP_ERR_MEM_LOCATION;
        return;
    }
    if (sdp_mem_num_dims(grid) != 2 || sdp_mem_num_dims(subgrid) != 2)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    if (!need_gpu(status)) return;
    Staged g, s;
    g.init(grid, status);
    s.init(subgrid, status);
    if (*status) return;
    const int64_t gu = sdp_mem_shape_dim(grid, 0);
    const int64_t gv = sdp_mem_shape_dim(grid, 1);
    const int64_t su = sdp_mem_shape_dim(subgrid, 0);
    const int64_t sv = sdp_mem_shape_dim(subgrid, 1);
    const dim3 blocks(blocks_of(sv), (unsigned)su);
    const int cplx = is_complex_type(tg) ? 1 : 0;
    if (su > 0 && sv > 0)
    {
        if (is_double_type(tg))
            k_subgrid_add<double><<<blocks, 256>>>(
                    (double*)sdp_mem_data(g.dev), gu, gv,
                    (const double*)sdp_mem_data(s.dev), su, sv, offset_u,
                    offset_v, factor, cplx);
        else
            k_subgrid_add<float><<<blocks, 256>>>(
                    (float*)sdp_mem_data(g.dev), gu, gv,
                    (const float*)sdp_mem_data(s.dev), su, sv, offset_u,
                    offset_v, factor, cplx);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    g.write_back(status);
}

void sdp_gridder_subgrid_cut_out(const sdp_Mem* grid, int offset_u,
        int offset_v, sdp_Mem* subgrid, sdp_Error* status)
{
    if (*status) return;
    const sdp_MemType tg = sdp_mem_type(grid);
    if (tg != sdp_mem_type(subgrid) || any_kind(tg) < 0)
    {
        SDP_LOG_ERROR("Unsupported grid or sub-grid data type");
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (sdp_mem_location(grid) != sdp_mem_location(subgrid))
    {
        SDP_LOG_ERROR("All arrays must be in the same memory space");
        *status = SDP_ERR_MEM_LOCATION;
        return;
    }
    if (sdp_mem_num_dims(grid) != 2 || sdp_mem_num_dims(subgrid) != 2)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    if (!need_gpu(status)) return;
    Staged g, s;
    g.init(grid, status);
    s.init(subgrid, status);
    if (*status) return;
    const int64_t gu = sdp_mem_shape_dim(grid, 0);
    const int64_t gv = sdp_mem_shape_dim(grid, 1);
    const int64_t su = sdp_mem_shape_dim(subgrid, 0);
    const int64_t sv = sdp_mem_shape_dim(subgrid, 1);
    const dim3 blocks(blocks_of(sv), (unsigned)su);
    const int cplx = is_complex_type(tg) ? 1 : 0;
    if (su > 0 && sv > 0)
    {
        if (is_double_type(tg))
            k_subgrid_cut_out<double><<<blocks, 256>>>(
                    (const double*)sdp_mem_data(g.dev), gu, gv,
                    (double*)sdp_mem_data(s.dev), su, sv, offset_u, offset_v,
                    cplx);
        else
            k_subgrid_cut_out<float><<<blocks, 256>>>(
                    (const float*)sdp_mem_data(g.dev), gu, gv,
                    (float*)sdp_mem_data(s.dev), su, sv, offset_u, offset_v,
                    cplx);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    s.write_back(status);
}

void sdp_gridder_sum_diff(const sdp_Mem* a, const sdp_Mem* b,
        int64_t* result, int64_t start_row, int64_t end_row,
        sdp_Error* status)
{
    if (*status) return;
    *result = 0;
    if (start_row < 0 || end_row < 0)
    {
        start_row = 0;
        end_row = sdp_mem_shape_dim(a, 0);
    }
    if (sdp_mem_type(a) != SDP_MEM_INT || sdp_mem_type(b) != SDP_MEM_INT)
    {
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (sdp_mem_shape_dim(a, 0) != sdp_mem_shape_dim(b, 0) ||
            sdp_mem_location(a) != sdp_mem_location(b))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    if (!need_gpu(status)) return;
    Staged da, db;
    da.init(a, status);
    db.init(b, status);
    unsigned long long* d_out = nullptr;
    SDP_HIP_CHECK(hipMalloc(&d_out, sizeof(*d_out)), status);
    if (*status) return;
    SDP_HIP_CHECK(hipMemsetAsync(d_out, 0, sizeof(*d_out), 0), status);
    if (end_row > start_row)
    {
        const unsigned blocks = std::min<unsigned>(1024,
                blocks_of(end_row - start_row));
        k_sum_diff<<<blocks, 256>>>((const int*)sdp_mem_data(da.dev),
                (const int*)sdp_mem_data(db.dev), start_row, end_row, d_out);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    unsigned long long h = 0;
    SDP_HIP_CHECK(hipMemcpy(&h, d_out, sizeof(h), hipMemcpyDeviceToHost),
            status);
    (void)hipFree(d_out);
    *result = (int64_t)h;
}

void sdp_gridder_uvw_bounds_all(const sdp_Mem* uvws, double freq0_hz,
        double dfreq_hz, const sdp_Mem* start_chs, const sdp_Mem* end_chs,
        double uvw_min[3], double uvw_max[3], sdp_Error* status)
{
    if (*status) return;
    for (int j = 0; j < 3; ++j)
    {
        uvw_min[j] = INFINITY;
        uvw_max[j] = -INFINITY;
    }
    const sdp_MemType t = sdp_mem_type(uvws);
    if (t != SDP_MEM_DOUBLE && t != SDP_MEM_FLOAT)
    {
        SDP_LOG_ERROR("Unsupported (u,v,w) data type");
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (sdp_mem_type(start_chs) != SDP_MEM_INT ||
            sdp_mem_type(end_chs) != SDP_MEM_INT)
    {
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (!need_gpu(status)) return;
    Staged u, s, e;
    u.init(uvws, status);
    s.init(start_chs, status);
    e.init(end_chs, status);
    if (*status) return;
    const int64_t rows = sdp_mem_shape_dim(uvws, 0);
    if (t == SDP_MEM_DOUBLE)
        uvw_bounds_dev<double>((const double*)sdp_mem_data(u.dev), rows,
                freq0_hz, dfreq_hz, (const int*)sdp_mem_data(s.dev),
                (const int*)sdp_mem_data(e.dev), uvw_min, uvw_max, status);
    else
        uvw_bounds_dev<float>((const float*)sdp_mem_data(u.dev), rows,
                freq0_hz, dfreq_hz, (const int*)sdp_mem_data(s.dev),
                (const int*)sdp_mem_data(e.dev), uvw_min, uvw_max, status);
}

static void clamp_impl(const sdp_Mem* uvws, int dim, int ndims, double f0,
        double df, const sdp_Mem* s_in, const sdp_Mem* e_in, double min0,
        double max0, double min1, double max1, sdp_Mem* s_out,
        sdp_Mem* e_out, int64_t r0, int64_t r1, sdp_Error* status)
{
    if (*status) return;
    if (r0 < 0 || r1 < 0)
    {
        r0 = 0;
        r1 = sdp_mem_shape_dim(uvws, 0);
    }
    const sdp_MemType t = sdp_mem_type(uvws);
    if (t != SDP_MEM_DOUBLE && t != SDP_MEM_FLOAT)
    {
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    if (sdp_mem_type(s_in) != SDP_MEM_INT || sdp_mem_type(e_in) != SDP_MEM_INT
            || sdp_mem_type(s_out) != SDP_MEM_INT ||
            sdp_mem_type(e_out) != SDP_MEM_INT)
    {
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    const sdp_MemLocation loc = sdp_mem_location(uvws);
    if (sdp_mem_location(s_in) != loc || sdp_mem_location(e_in) != loc ||
            sdp_mem_location(s_out) != loc || sdp_mem_location(e_out) != loc)
    {
        SDP_LOG_ERROR("All arrays must be in the same memory space");
        *status = SDP_ERR_MEM_LOCATION;
        return;
    }
    if (dim < 0 || dim + ndims > 3)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    if (!need_gpu(status)) return;
    Staged u, si, ei, so, eo;
    u.init(uvws, status);
    si.init(s_in, status);
    ei.init(e_in, status);
    so.init(s_out, status);
    eo.init(e_out, status);
    if (*status) return;
    if (r1 > r0)
    {
        const unsigned blocks = blocks_of(r1 - r0);
        if (t == SDP_MEM_DOUBLE)
            k_clamp<double><<<blocks, 256>>>(
                    (const double*)sdp_mem_data(u.dev), dim, ndims, f0, df,
                    (const int*)sdp_mem_data(si.dev),
                    (const int*)sdp_mem_data(ei.dev), min0, max0, min1, max1,
                    (int*)sdp_mem_data(so.dev), (int*)sdp_mem_data(eo.dev),
                    r0, r1);
        else
            k_clamp<float><<<blocks, 256>>>(
                    (const float*)sdp_mem_data(u.dev), dim, ndims, f0, df,
                    (const int*)sdp_mem_data(si.dev),
                    (const int*)sdp_mem_data(ei.dev), min0, max0, min1, max1,
                    (int*)sdp_mem_data(so.dev), (int*)sdp_mem_data(eo.dev),
                    r0, r1);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    so.write_back(status);
    eo.write_back(status);
}

void sdp_gridder_clamp_channels_single(const sdp_Mem* uvws, const int dim,
        const double freq0_hz, const double dfreq_hz,
        const sdp_Mem* start_ch_in, const sdp_Mem* end_ch_in,
        const double min_u, const double max_u, sdp_Mem* start_ch_out,
        sdp_Mem* end_ch_out, int64_t start_row, int64_t end_row,
        sdp_Error* status)
{
    clamp_impl(uvws, dim, 1, freq0_hz, dfreq_hz, start_ch_in, end_ch_in,
            min_u, max_u, 0.0, 0.0, start_ch_out, end_ch_out, start_row,
            end_row, status);
}

void sdp_gridder_clamp_channels_uv(const sdp_Mem* uvws,
        const double freq0_hz, const double dfreq_hz,
        const sdp_Mem* start_ch_in, const sdp_Mem* end_ch_in,
        const double min_u, const double max_u, const double min_v,
        const double max_v, sdp_Mem* start_ch_out, sdp_Mem* end_ch_out,
        int64_t start_row, int64_t end_row, sdp_Error* status)
{
    clamp_impl(uvws, 0, 2, freq0_hz, dfreq_hz, start_ch_in, end_ch_in,
            min_u, max_u, min_v, max_v, start_ch_out, end_ch_out, start_row,
            end_row, status);
}

} // extern "C"
