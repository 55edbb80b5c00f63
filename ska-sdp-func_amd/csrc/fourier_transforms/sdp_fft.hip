// sdp_fft_* C ABI on rocFFT (include/ska-sdp-func/fourier_transforms/
// sdp_fft.h), replacing the reference's cuFFT / PocketFFT wrapper
// (src/ska-sdp-func/fourier_transforms/sdp_fft.cpp:295-1191, sdp_fft.cu).
//
// Conventions kept from the reference: C2C / Z2Z only, unnormalised in both
// directions (inverse = +i exponent), 1-, 2- or 3-D transforms, a batch over
// the first (slowest) dimension when the arrays have one dimension more than
// the transform, C-contiguous arrays, and exec() requires arrays matching
// the ones the plan was created with (sdp_fft.cpp:883-921).
//
// MI355X-specific: rocFFT plans are placement-specific, so the in-place and
// out-of-place plans are created on first use and cached in the handle
// (exec_shift always runs in place). Host arrays are staged through HBM:
// the transform itself always runs on the GPU (there is no CPU FFT here).
#include <algorithm>
#include <map>
#include <mutex>
#include <cstdlib>
#include <cstring>

#include <rocfft/rocfft.h>

#include "ska-sdp-func/fourier_transforms/sdp_fft.h"
#include "ska-sdp-func/fourier_transforms/sdp_fft_padded_size.h"
#include "ska-sdp-func/utility/sdp_logging.h"
#include "../grid_data/es_fft.h"
#include "../utility/sdp_hip.h"

struct sdp_Fft
{
    sdp_Mem* input;          // aliases of the creation arrays
    sdp_Mem* output;
    int num_dims;
    int64_t batch;
    int is_forward;
    int dbl;
    size_t lengths[3];       // rocFFT order: fastest first
    rocfft_plan plan[2];     // [0] in place, [1] out of place
    rocfft_execution_info info;
    void* work;
    size_t work_bytes;
};

namespace {

bool rocfft_ready(sdp_Error* status)
{
    static int state = 0;    // rocfft_setup is idempotent; call once
    if (state == 0) state = (rocfft_setup() == rocfft_status_success) ? 1 : -1;
    if (state < 0)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("rocfft_setup failed");
        return false;
    }
    return true;
}

// sdp_fft.cpp:295-356.
void check_params(const sdp_Mem* input, const sdp_Mem* output,
        int32_t num_dims_fft, sdp_Error* status)
{
    if (*status) return;
    if (sdp_mem_is_read_only(output))
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("Output array is read-only");
        return;
    }
    if (sdp_mem_location(input) != sdp_mem_location(output))
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Input and output arrays must be in the same location");
        return;
    }
    if (sdp_mem_num_dims(input) != sdp_mem_num_dims(output))
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("Input and output arrays must have the same "
                "number of dimensions");
        return;
    }
    if (!sdp_mem_is_c_contiguous(input) || !sdp_mem_is_c_contiguous(output))
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("All arrays must be C-contiguous");
        return;
    }
    if (sdp_mem_is_complex(input) && sdp_mem_is_complex(output))
    {
        for (int32_t i = 0; i < sdp_mem_num_dims(input); ++i)
        {
            if (sdp_mem_shape_dim(input, i) != sdp_mem_shape_dim(output, i))
            {
                *status = SDP_ERR_RUNTIME;
                SDP_LOG_ERROR("Inconsistent array dimension sizes");
                return;
            }
        }
    }
    else
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data types");
        return;
    }
    if (sdp_mem_type(input) != sdp_mem_type(output))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data types");
        return;
    }
    if (num_dims_fft != sdp_mem_num_dims(input) &&
            num_dims_fft != sdp_mem_num_dims(input) - 1)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("Number of FFT dimensions must be equal to "
                "or one smaller than the number of array dimensions");
        return;
    }
    if (num_dims_fft < 1 || num_dims_fft > 3)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Only 1-, 2- and 3-D FFTs are supported");
    }
}

rocfft_plan make_plan(const sdp_Fft* fft, bool in_place, sdp_Error* status)
{
    rocfft_plan plan = nullptr;
    const rocfft_status e = rocfft_plan_create(&plan,
            in_place ? rocfft_placement_inplace : rocfft_placement_notinplace,
            fft->is_forward ? rocfft_transform_type_complex_forward :
                    rocfft_transform_type_complex_inverse,
            fft->dbl ? rocfft_precision_double : rocfft_precision_single,
            (size_t)fft->num_dims, fft->lengths, (size_t)fft->batch, nullptr);
    if (e != rocfft_status_success)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("rocfft_plan_create error (code %d)", (int)e);
        return nullptr;
    }
    return plan;
}

bool ensure_plan(sdp_Fft* fft, bool in_place, sdp_Error* status)
{
    rocfft_plan& p = fft->plan[in_place ? 0 : 1];
    if (p) return true;
    p = make_plan(fft, in_place, status);
    if (!p) return false;
    size_t w = 0;
    rocfft_plan_get_work_buffer_size(p, &w);
    if (w > fft->work_bytes)
    {
        if (fft->work) (void)hipFree(fft->work);
        fft->work = nullptr;
        fft->work_bytes = 0;
        SDP_HIP_CHECK(hipMalloc(&fft->work, w), status);
        if (*status) return false;
        fft->work_bytes = w;
        rocfft_execution_info_set_work_buffer(fft->info, fft->work, w);
    }
    return true;
}

void exec_device(sdp_Fft* fft, void* in, void* out, sdp_Error* status)
{
    const bool in_place = (in == out);
    if (!ensure_plan(fft, in_place, status)) return;
    rocfft_execution_info_set_stream(fft->info, 0);
    void* ibuf[1] = {in};
    void* obuf[1] = {out};
    const rocfft_status e = rocfft_execute(fft->plan[in_place ? 0 : 1],
            ibuf, in_place ? nullptr : obuf, fft->info);
    if (e != rocfft_status_success)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("rocfft_execute error (code %d)", (int)e);
    }
}

// (-1)^(ix + iy) on a [nx][ny] complex array (sdp_fft.cu:11-19).
template<typename T>
__global__ void k_fft_phase(T* data, int64_t nx, int64_t ny)
{
    const int64_t iy = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (iy >= ny) return;
    // Rows stride over the y-grid (capped at 65535 blocks by the host).
    for (int64_t ix = blockIdx.y; ix < nx; ix += gridDim.y)
    {
        if (((ix + iy) & 1) == 0) continue;
        T* p = data + 2 * (ix * ny + iy);
        p[0] = -p[0];
        p[1] = -p[1];
    }
}

// data *= factor (sdp_fft.cu:21-29), factor in double converted to T as
// complex<T> *= double does on the host.
template<typename T>
__global__ void k_fft_norm(T* data, int64_t n, double factor)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= 2 * n) return;
    data[i] = (T)((double)data[i] * factor);
}

// A device copy of a host array (or the array itself on the GPU).
struct DevArray
{
    sdp_Mem* mem = nullptr;
    sdp_Mem* src = nullptr;
    bool staged = false;

    void init(sdp_Mem* m, sdp_Error* status)
    {
        src = m;
        if (*status || !m) return;
        if (sdp_mem_location(m) == SDP_MEM_GPU)
        {
            mem = m;
            return;
        }
        mem = sdp_mem_create_copy(m, SDP_MEM_GPU, status);
        staged = true;
    }

    void write_back(sdp_Error* status)
    {
        if (staged && !*status)
            sdp_mem_copy_contents(src, mem, 0, 0, sdp_mem_num_elements(src),
                    status);
    }

    ~DevArray()
    {
        if (staged) sdp_mem_free(mem);
    }
};

bool have_gpu(sdp_Error* status)
{
    if (sdp_hip::device_available()) return true;
    *status = SDP_ERR_MEM_LOCATION;
    SDP_LOG_ERROR("No GPU available for the FFT");
    return false;
}

void fft_exec_mem(sdp_Fft* fft, sdp_Mem* input, sdp_Mem* output,
        sdp_Error* status)
{
    if (*status) return;
    if (!have_gpu(status)) return;
    if (sdp_mem_location(input) == SDP_MEM_GPU)
    {
        exec_device(fft, sdp_mem_data(input), sdp_mem_data(output), status);
        return;
    }
    // Host arrays: one staging buffer in place when input == output.
    DevArray in, out;
    in.init(input, status);
    if (sdp_mem_data(output) == sdp_mem_data(input))
    {
        exec_device(fft, sdp_mem_data(in.mem), sdp_mem_data(in.mem), status);
        in.write_back(status);
        return;
    }
    out.init(output, status);
    if (*status) return;
    exec_device(fft, sdp_mem_data(in.mem), sdp_mem_data(out.mem), status);
    out.write_back(status);
}

} // namespace

extern "C" {

sdp_Fft* sdp_fft_create(const sdp_Mem* input, const sdp_Mem* output,
        int32_t num_dims_fft, int32_t is_forward, sdp_Error* status)
{
    if (*status) return nullptr;
    check_params(input, output, num_dims_fft, status);
    if (*status) return nullptr;
    const sdp_MemLocation loc = sdp_mem_location(input);
    if (loc != SDP_MEM_GPU && loc != SDP_MEM_CPU)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Unsupported FFT location");
        return nullptr;
    }
    if (!have_gpu(status) || !rocfft_ready(status)) return nullptr;
    sdp_Fft* fft = (sdp_Fft*)calloc(1, sizeof(sdp_Fft));
    fft->input = sdp_mem_create_alias(input);
    fft->output = sdp_mem_create_alias(output);
    fft->num_dims = num_dims_fft;
    fft->is_forward = is_forward;
    fft->dbl = sdp_mem_type(input) == SDP_MEM_COMPLEX_DOUBLE;
    const int32_t nd = sdp_mem_num_dims(input);
    fft->batch = (nd != num_dims_fft) ? sdp_mem_shape_dim(input, 0) : 1;
    for (int i = 0; i < num_dims_fft; ++i)
        fft->lengths[i] = (size_t)sdp_mem_shape_dim(input, nd - 1 - i);
    rocfft_execution_info_create(&fft->info);
    // The plan for the creation arrays' placement is made now, so that
    // unsupported sizes fail at creation as they do with cuFFT.
    const bool in_place = sdp_mem_data_const(input) ==
            sdp_mem_data_const(output);
    if (!ensure_plan(fft, in_place, status))
    {
        sdp_fft_free(fft);
        return nullptr;
    }
    return fft;
}

void sdp_fft_exec(sdp_Fft* fft, sdp_Mem* input, sdp_Mem* output,
        sdp_Error* status)
{
    if (*status || !fft || !input || !output) return;
    check_params(input, output, fft->num_dims, status);
    if (*status) return;
    if (!sdp_mem_is_matching(fft->input, input, 1) ||
            !sdp_mem_is_matching(fft->output, output, 1))
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("Arrays do not match those used for FFT plan creation");
        return;
    }
    fft_exec_mem(fft, input, output, status);
}

void sdp_fft_exec_shift(sdp_Fft* fft, sdp_Mem* data, int norm,
        sdp_Error* status)
{
    if (*status) return;
    sdp_fft_phase(data, status);
    sdp_fft_exec(fft, data, data, status);
    sdp_fft_phase(data, status);
    if (norm) sdp_fft_norm(data, status);
}

void sdp_fft_free(sdp_Fft* fft)
{
    if (!fft) return;
    for (int i = 0; i < 2; ++i)
        if (fft->plan[i]) rocfft_plan_destroy(fft->plan[i]);
    if (fft->info) rocfft_execution_info_destroy(fft->info);
    if (fft->work) (void)hipFree(fft->work);
    sdp_mem_ref_dec(fft->input);
    sdp_mem_ref_dec(fft->output);
    free(fft);
}

void sdp_fft_norm(sdp_Mem* data, sdp_Error* status)
{
    if (*status || !data) return;
    const sdp_MemType t = sdp_mem_type(data);
    if (t != SDP_MEM_COMPLEX_FLOAT && t != SDP_MEM_COMPLEX_DOUBLE)
    {
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    const sdp_MemLocation loc = sdp_mem_location(data);
    if (loc != SDP_MEM_CPU && loc != SDP_MEM_GPU)
    {
        *status = SDP_ERR_MEM_LOCATION;
        return;
    }
    if (sdp_mem_num_dims(data) != 2 || !sdp_mem_is_c_contiguous(data))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("sdp_fft_norm: data must be a 2-D C-contiguous array");
        return;
    }
    if (!have_gpu(status)) return;
    const int64_t nx = sdp_mem_shape_dim(data, 0);
    const int64_t ny = sdp_mem_shape_dim(data, 1);
    const int64_t n = nx * ny;
    // sdp_fft.cpp:977-990: factor = 1.0 / (num_x * num_y) in int arithmetic.
    const double factor = 1.0 / (double)(int)(nx * ny);
    DevArray d;
    d.init(data, status);
    if (*status) return;
    const unsigned blocks = sdp_hip::blocks_for(2 * n, 256);
    if (t == SDP_MEM_COMPLEX_FLOAT)
        k_fft_norm<float><<<blocks, 256>>>((float*)sdp_mem_data(d.mem), n,
                factor);
    else
        k_fft_norm<double><<<blocks, 256>>>((double*)sdp_mem_data(d.mem), n,
                factor);
    SDP_HIP_CHECK_LAUNCH(status);
    d.write_back(status);
}

void sdp_fft_phase(sdp_Mem* data, sdp_Error* status)
{
    if (*status || !data) return;
    const sdp_MemType t = sdp_mem_type(data);
    if (t != SDP_MEM_COMPLEX_FLOAT && t != SDP_MEM_COMPLEX_DOUBLE)
    {
        *status = SDP_ERR_DATA_TYPE;
        return;
    }
    const sdp_MemLocation loc = sdp_mem_location(data);
    if (loc != SDP_MEM_CPU && loc != SDP_MEM_GPU)
    {
        *status = SDP_ERR_MEM_LOCATION;
        return;
    }
    const int nd = sdp_mem_num_dims(data);
    if ((nd != 1 && nd != 2) || !sdp_mem_is_c_contiguous(data))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("sdp_fft_phase: data must be a 1-D or 2-D "
                "C-contiguous array");
        return;
    }
    if (!have_gpu(status)) return;
    const int64_t nx = (nd == 2) ? sdp_mem_shape_dim(data, 0) : 1;
    const int64_t ny = sdp_mem_shape_dim(data, nd - 1);
    DevArray d;
    d.init(data, status);
    if (*status) return;
    const dim3 blocks(sdp_hip::blocks_for(ny, 256),
            (unsigned)std::min<int64_t>(nx, 65535));
    if (t == SDP_MEM_COMPLEX_FLOAT)
        k_fft_phase<float><<<blocks, 256>>>((float*)sdp_mem_data(d.mem), nx,
                ny);
    else
        k_fft_phase<double><<<blocks, 256>>>((double*)sdp_mem_data(d.mem),
                nx, ny);
    SDP_HIP_CHECK_LAUNCH(status);
    d.write_back(status);
}

// sdp_fft_padded_size.cpp:87-126: the smallest even m >= ceil(n * factor)
// whose half is 11-smooth (the reference walks a min-heap of 2 x products
// of 2, 3, 5, 7, 11; this enumerates candidates directly).
void sdp_fft_2d_inplace_permuted(sdp_Mem* data, int is_forward,
        sdp_Error* status)
{
    if (*status) return;
    const int64_t G = sdp_mem_num_dims(data) == 2 ?
            sdp_mem_shape_dim(data, 0) : 0;
    if (sdp_mem_type(data) != SDP_MEM_COMPLEX_FLOAT ||
            sdp_mem_location(data) != SDP_MEM_GPU ||
            sdp_mem_shape_dim(data, 1) != G || G > 16384 ||
            !sdp_es::fused_fft_supported((int)G) ||
            !sdp_mem_is_c_contiguous(data))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("sdp_fft_2d_inplace_permuted: a square complex-float "
                "GPU array, side a power of two in [1024, 16384]");
        return;
    }
    // Twiddle tables are built once per (device, grid size) and kept for the
    // life of the process (at most five sizes, 1024..16384, per device; a
    // per-plane caller pays no allocation). The tables live in the memory of
    // the device current at creation, so the key carries the device: a call
    // on another GPU with the same G gets its own tables. The transform runs
    // on the null stream, as the other sdp_fft_* kernels here, and returns
    // when it is complete.
    static std::mutex tw_lock;
    static std::map<std::pair<int, int>, sdp_es::FftTwiddles> tw_cache;
    int e = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
    {
        *status = SDP_ERR_RUNTIME;
        return;
    }
    sdp_es::FftTwiddles tw;
    {
        std::lock_guard<std::mutex> guard(tw_lock);
        const auto key = std::make_pair(dev, (int)G);
        auto it = tw_cache.find(key);
        if (it == tw_cache.end())
        {
            e = sdp_es::fft_twiddles_create((int)G, &tw);
            if (!e) tw_cache.emplace(key, tw);
        }
        else
        {
            tw = it->second;
        }
    }
    if (!e)
        e = sdp_es::fft2d_inplace_permuted((float*)sdp_mem_data(data),
                (int)G, is_forward != 0, tw, 0);
    if (!e) e = (int)hipStreamSynchronize(0) ? SDP_ERR_RUNTIME : 0;
    if (e) *status = (sdp_Error)e;
}

int sdp_fft_permuted_n2(int grid_size)
{
    return sdp_es::fft_perm_n2(grid_size);
}

int sdp_fft_padded_size(int n, double padding_factor)
{
    const long long target = (long long)ceil(n * padding_factor);
    long long m = target < 2 ? 2 : target + (target & 1);
    for (;; m += 2)
    {
        long long r = m / 2;
        const int primes[] = {2, 3, 5, 7, 11};
        for (int p : primes)
            while (r % p == 0) r /= p;
        if (r == 1) return (int)m;
    }
}

} // extern "C"
