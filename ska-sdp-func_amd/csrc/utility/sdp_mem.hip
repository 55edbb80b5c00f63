// sdp_Mem: tensor handle with the reference's C ABI
// (src/ska-sdp-func/utility/sdp_mem.h / sdp_mem.cpp), backed by HIP on MI355X.
//
// Layout of the handle follows what the reference stores (sdp_mem.cpp:20-33):
// element type, location, byte strides, ownership, read-only flag and a plain
// (non-atomic) reference count. GPU memory is hipMalloc'ed on the current
// device; copies use hipMemcpy with hipMemcpyDefault (unified addressing).
#include <complex>
#include <cstdlib>
#include <cstring>

#include "ska-sdp-func/utility/sdp_mem.h"
#include "sdp_hip.h"

struct sdp_Mem
{
    sdp_MemType type;
    sdp_MemLocation location;
    int32_t is_c_contiguous;
    int32_t is_owner;
    int32_t is_read_only;
    int32_t num_dims;
    int64_t num_elements;
    int32_t ref_count;
    int64_t* shape;
    int64_t* stride;   // bytes
    void* data;
};

struct sdp_CudaStream
{
    hipStream_t stream;
};

namespace sdp_hip {

bool device_available()
{
    static int cached = -1;
    if (cached < 0)
    {
        int n = 0;
        cached = (hipGetDeviceCount(&n) == hipSuccess && n > 0) ? 1 : 0;
        (void)hipGetLastError();
    }
    return cached == 1;
}

} // namespace sdp_hip

namespace {

void mem_alloc(sdp_Mem* mem, sdp_Error* status)
{
    mem->is_owner = 1;
    const size_t bytes = (size_t)mem->num_elements *
            (size_t)sdp_mem_type_size(mem->type);
    if (*status || bytes == 0) return;
    if (mem->location == SDP_MEM_CPU)
    {
        mem->data = calloc(bytes, 1);
        if (!mem->data)
        {
            *status = SDP_ERR_MEM_ALLOC_FAILURE;
            SDP_LOG_CRITICAL("Host memory allocation failure "
                    "(requested %zu bytes)", bytes);
        }
    }
    else if (mem->location == SDP_MEM_GPU)
    {
        if (!sdp_hip::device_available())
        {
            *status = SDP_ERR_MEM_LOCATION;
            SDP_LOG_ERROR("Cannot allocate GPU memory: no HIP device");
            return;
        }
        const hipError_t err = hipMalloc(&mem->data, bytes);
        if (err != hipSuccess || !mem->data)
        {
            mem->data = nullptr;
            *status = SDP_ERR_MEM_ALLOC_FAILURE;
            SDP_LOG_CRITICAL("GPU memory allocation failure "
                    "(requested %zu bytes): %s", bytes, hipGetErrorString(err));
        }
    }
    else
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Unsupported memory location");
    }
}

template<typename T>
__global__ void k_scale_real(T* data, int64_t n, double value)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) data[i] *= value;
}

template<typename T>
__global__ void k_scale_real_complex(T* data, int64_t n, double value)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) data[2 * i] *= value;
}

// Strided set (up to 3 dims), element type T (complex: real part = value).
template<typename T, int NCOMP>
__global__ void k_set_value(char* base, int64_t n0, int64_t n1, int64_t n2,
        int64_t s0, int64_t s1, int64_t s2, T value)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = n0 * n1 * n2;
    if (i >= total) return;
    const int64_t i2 = i % n2, i1 = (i / n2) % n1, i0 = i / (n1 * n2);
    T* p = (T*)(base + i0 * s0 + i1 * s1 + i2 * s2);
    p[0] = value;
    if (NCOMP == 2) p[1] = T(0);
}

template<typename T, int NCOMP>
void set_value_cpu(sdp_Mem* mem, T value, const int64_t n[3],
        const int64_t s[3])
{
    char* base = (char*)mem->data;
    for (int64_t i0 = 0; i0 < n[0]; ++i0)
        for (int64_t i1 = 0; i1 < n[1]; ++i1)
            for (int64_t i2 = 0; i2 < n[2]; ++i2)
            {
                T* p = (T*)(base + i0 * s[0] + i1 * s[1] + i2 * s[2]);
                p[0] = value;
                if (NCOMP == 2) p[1] = T(0);
            }
}

} // namespace

extern "C" {

int64_t sdp_mem_type_size(sdp_MemType type)
{
    switch (type)
    {
    case SDP_MEM_CHAR: return 1;
    case SDP_MEM_INT: return sizeof(int);
    case SDP_MEM_FLOAT: return sizeof(float);
    case SDP_MEM_DOUBLE: return sizeof(double);
    case SDP_MEM_COMPLEX_FLOAT: return 2 * sizeof(float);
    case SDP_MEM_COMPLEX_DOUBLE: return 2 * sizeof(double);
    default: return 0;
    }
}

const char* sdp_mem_type_name(sdp_MemType type)
{
    switch (type)
    {
    case SDP_MEM_VOID: return "void";
    case SDP_MEM_CHAR: return "char";
    case SDP_MEM_INT: return "int";
    case SDP_MEM_FLOAT: return "float";
    case SDP_MEM_DOUBLE: return "double";
    case SDP_MEM_COMPLEX_FLOAT: return "complex float";
    case SDP_MEM_COMPLEX_DOUBLE: return "complex double";
    default: return "unknown";
    }
}

const char* sdp_mem_location_name(sdp_MemLocation location)
{
    switch (location)
    {
    case SDP_MEM_CPU: return "CPU";
    case SDP_MEM_GPU: return "GPU";
    default: return "unknown";
    }
}

sdp_Mem* sdp_mem_create_wrapper(void* data, sdp_MemType type,
        sdp_MemLocation location, int32_t num_dims, const int64_t* shape,
        const int64_t* stride, sdp_Error* status)
{
    sdp_Mem* mem = (sdp_Mem*)calloc(1, sizeof(sdp_Mem));
    mem->data = data;
    mem->ref_count = 1;
    mem->type = type;
    mem->location = location;
    mem->num_dims = num_dims;
    mem->is_c_contiguous = 1;
    if (type == SDP_MEM_VOID) return mem;   // empty wrapper (Python Mem())
    const int64_t esize = sdp_mem_type_size(type);
    if (esize <= 0)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_CRITICAL("Unsupported data type");
        return mem;
    }
    mem->num_elements = 1;
    if (num_dims <= 0) return mem;   // 0-d tensor = scalar
    mem->shape = (int64_t*)calloc(num_dims, sizeof(int64_t));
    mem->stride = (int64_t*)calloc(num_dims, sizeof(int64_t));
    for (int32_t i = num_dims - 1; i >= 0; --i)
    {
        mem->shape[i] = shape[i];
        mem->stride[i] = stride ? stride[i] : mem->num_elements * esize;
        mem->num_elements *= shape[i];
    }
    int64_t expect = esize;
    for (int32_t i = num_dims - 1; i >= 0; --i)
    {
        if (mem->stride[i] != expect) mem->is_c_contiguous = 0;
        expect *= shape[i];
    }
    return mem;
}

sdp_Mem* sdp_mem_create(sdp_MemType type, sdp_MemLocation location,
        int32_t num_dims, const int64_t* shape, sdp_Error* status)
{
    sdp_Mem* mem = sdp_mem_create_wrapper(nullptr, type, location, num_dims,
            shape, nullptr, status);
    mem_alloc(mem, status);
    return mem;
}

sdp_Mem* sdp_mem_create_wrapper_for_slice(const sdp_Mem* src,
        const int64_t* slice_offsets, const int32_t num_dims_slice,
        const int64_t* slice_shape, sdp_Error* status)
{
    if (*status) return nullptr;
    if (num_dims_slice > src->num_dims)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Slice has more dimensions (%d) than source (%d)",
                num_dims_slice, src->num_dims);
        return nullptr;
    }
    int64_t offset_bytes = 0;
    for (int32_t i = 0; i < src->num_dims; ++i)
    {
        if (slice_offsets[i] < 0 || slice_offsets[i] >= src->shape[i])
        {
            *status = SDP_ERR_INVALID_ARGUMENT;
            SDP_LOG_ERROR("Slice offset %lld out of range in dimension %d",
                    (long long)slice_offsets[i], i);
            return nullptr;
        }
        offset_bytes += slice_offsets[i] * src->stride[i];
    }
    int64_t* strides = (int64_t*)calloc(num_dims_slice > 0 ? num_dims_slice : 1,
            sizeof(int64_t));
    for (int32_t i = 0; i < num_dims_slice; ++i)
    {
        // Slice dimensions align with the trailing source dimensions.
        const int32_t src_dim = src->num_dims - num_dims_slice + i;
        if (slice_offsets[src_dim] + slice_shape[i] > src->shape[src_dim])
        {
            *status = SDP_ERR_INVALID_ARGUMENT;
            SDP_LOG_ERROR("Slice shape too large in dimension %d", i);
            free(strides);
            return nullptr;
        }
        strides[i] = src->stride[src_dim];
    }
    sdp_Mem* mem = sdp_mem_create_wrapper((char*)src->data + offset_bytes,
            src->type, src->location, num_dims_slice, slice_shape, strides,
            status);
    free(strides);
    return mem;
}

sdp_Mem* sdp_mem_create_alias(const sdp_Mem* src)
{
    sdp_Error status = SDP_SUCCESS;
    return sdp_mem_create_wrapper(src->data, src->type, src->location,
            src->num_dims, src->shape, src->stride, &status);
}

sdp_Mem* sdp_mem_create_copy(const sdp_Mem* src, sdp_MemLocation location,
        sdp_Error* status)
{
    sdp_Mem* mem = sdp_mem_create_wrapper(nullptr, src->type, location,
            src->num_dims, src->shape, src->stride, status);
    mem_alloc(mem, status);
    sdp_mem_copy_contents(mem, src, 0, 0, src->num_elements, status);
    return mem;
}

void sdp_mem_clear_portion(sdp_Mem* mem, int64_t start_index,
        int64_t num_elements, sdp_Error* status)
{
    if (*status || !mem || num_elements == 0) return;
    const int64_t esize = sdp_mem_type_size(mem->type);
    char* p = (char*)mem->data + start_index * esize;
    const size_t bytes = (size_t)(num_elements * esize);
    if (mem->location == SDP_MEM_CPU)
    {
        memset(p, 0, bytes);
    }
    else if (mem->location == SDP_MEM_GPU)
    {
        SDP_HIP_CHECK(hipMemsetAsync(p, 0, bytes, 0), status);
    }
    else
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Unsupported memory location");
    }
}

void sdp_mem_clear_contents(sdp_Mem* mem, sdp_Error* status)
{
    if (*status || !mem || mem->num_elements == 0) return;
    sdp_mem_clear_portion(mem, 0, mem->num_elements, status);
}

static void copy_impl(sdp_Mem* dst, const sdp_Mem* src, int64_t offset_dst,
        int64_t offset_src, int64_t num_elements, hipStream_t stream,
        bool async, sdp_Error* status)
{
    if (*status || !dst || !src || !dst->data || !src->data) return;
    if (num_elements == 0) return;
    if (src->type != dst->type)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Cannot copy data between different types");
        return;
    }
    const int64_t esize = sdp_mem_type_size(src->type);
    const char* ps = (const char*)src->data + offset_src * esize;
    char* pd = (char*)dst->data + offset_dst * esize;
    const size_t bytes = (size_t)(num_elements * esize);
    if (src->location == SDP_MEM_CPU && dst->location == SDP_MEM_CPU)
    {
        memcpy(pd, ps, bytes);
        return;
    }
    if (!sdp_hip::device_available())
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("GPU copy requested but no HIP device is available");
        return;
    }
    const hipError_t err = async ?
            hipMemcpyAsync(pd, ps, bytes, hipMemcpyDefault, stream) :
            hipMemcpy(pd, ps, bytes, hipMemcpyDefault);
    if (err != hipSuccess)
    {
        *status = SDP_ERR_MEM_COPY_FAILURE;
        SDP_LOG_ERROR("hipMemcpy failed: %s", hipGetErrorString(err));
    }
}

void sdp_mem_copy_contents(sdp_Mem* dst, const sdp_Mem* src,
        int64_t offset_dst, int64_t offset_src, int64_t num_elements,
        sdp_Error* status)
{
    copy_impl(dst, src, offset_dst, offset_src, num_elements, 0, false,
            status);
}

void sdp_mem_copy_contents_async(sdp_Mem* dst, const sdp_Mem* src,
        int64_t offset_dst, int64_t offset_src, int64_t num_elements,
        sdp_CudaStream* stream, sdp_Error* status)
{
    copy_impl(dst, src, offset_dst, offset_src, num_elements,
            stream ? stream->stream : 0, true, status);
}

sdp_Mem* sdp_mem_convert_precision(const sdp_Mem* src,
        sdp_MemType output_type, sdp_Error* status)
{
    if (*status) return nullptr;
    if (!sdp_mem_is_c_contiguous(src))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Array must be C contiguous");
        return nullptr;
    }
    if (src->type == output_type)
    {
        return sdp_mem_create_copy(src, SDP_MEM_CPU, status);
    }
    sdp_Mem* tmp = nullptr;
    const sdp_Mem* in = src;
    if (src->location != SDP_MEM_CPU)
    {
        tmp = sdp_mem_create_copy(src, SDP_MEM_CPU, status);
        in = tmp;
    }
    sdp_Mem* out = sdp_mem_create(output_type, SDP_MEM_CPU, src->num_dims,
            src->shape, status);
    if (*status)
    {
        sdp_mem_free(tmp);
        return out;
    }
    const int64_t n = src->num_elements *
            (sdp_mem_is_complex(src) ? 2 : 1);
    const sdp_MemType a = src->type, b = output_type;
    if ((a & SDP_MEM_COMPLEX) != (b & SDP_MEM_COMPLEX))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Cannot convert between real and complex types");
    }
    else if ((a & SDP_MEM_DOUBLE) && (b & SDP_MEM_FLOAT))
    {
        const double* i_ = (const double*)in->data;
        float* o_ = (float*)out->data;
        for (int64_t i = 0; i < n; ++i) o_[i] = (float)i_[i];
    }
    else if ((a & SDP_MEM_FLOAT) && (b & SDP_MEM_DOUBLE))
    {
        const float* i_ = (const float*)in->data;
        double* o_ = (double*)out->data;
        for (int64_t i = 0; i < n; ++i) o_[i] = (double)i_[i];
    }
    else
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported precision conversion");
    }
    sdp_mem_free(tmp);
    return out;
}

void* sdp_mem_data(sdp_Mem* mem)
{
    return mem ? mem->data : nullptr;
}

const void* sdp_mem_data_const(const sdp_Mem* mem)
{
    return mem ? mem->data : nullptr;
}

void* sdp_mem_gpu_buffer(sdp_Mem* mem, sdp_Error* status)
{
    if (*status || !mem) return nullptr;
    if (mem->location != SDP_MEM_GPU && mem->type != SDP_MEM_VOID)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_CRITICAL("Requested buffer is not in GPU memory");
        return nullptr;
    }
    return &mem->data;
}

const void* sdp_mem_gpu_buffer_const(const sdp_Mem* mem, sdp_Error* status)
{
    if (*status || !mem) return nullptr;
    if (mem->location != SDP_MEM_GPU && mem->type != SDP_MEM_VOID)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_CRITICAL("Requested buffer is not in GPU memory");
        return nullptr;
    }
    return &mem->data;
}

void sdp_mem_free(sdp_Mem* mem)
{
    if (!mem) return;
    if (--mem->ref_count > 0) return;
    if (mem->is_owner && mem->data)
    {
        if (mem->location == SDP_MEM_CPU) free(mem->data);
        else if (mem->location == SDP_MEM_GPU) (void)hipFree(mem->data);
    }
    free(mem->shape);
    free(mem->stride);
    free(mem);
}

int32_t sdp_mem_is_c_contiguous(const sdp_Mem* mem)
{
    return (!mem || !mem->data) ? 0 : mem->is_c_contiguous;
}

int32_t sdp_mem_is_floating_point(const sdp_Mem* mem)
{
    if (!mem || !mem->data) return 0;
    return (mem->type & SDP_MEM_FLOAT) == SDP_MEM_FLOAT ||
            (mem->type & SDP_MEM_DOUBLE) == SDP_MEM_DOUBLE;
}

int32_t sdp_mem_is_complex(const sdp_Mem* mem)
{
    if (!mem || !mem->data) return 0;
    return (mem->type & SDP_MEM_COMPLEX) == SDP_MEM_COMPLEX;
}

int32_t sdp_mem_is_complex4(const sdp_Mem* mem)
{
    if (!sdp_mem_is_complex(mem)) return 0;
    const int32_t nd = mem->num_dims;
    return (nd > 1 && mem->shape[nd - 1] == 4) ||
            (nd > 2 && mem->shape[nd - 1] == 2 && mem->shape[nd - 2] == 2);
}

int32_t sdp_mem_is_double(const sdp_Mem* mem)
{
    if (!mem || !mem->data) return 0;
    return (mem->type & SDP_MEM_DOUBLE) == SDP_MEM_DOUBLE;
}

int32_t sdp_mem_is_matching(const sdp_Mem* mem1, const sdp_Mem* mem2,
        int32_t check_location)
{
    if (mem1->type != mem2->type) return 0;
    if (check_location && mem1->location != mem2->location) return 0;
    if (mem1->num_dims != mem2->num_dims) return 0;
    for (int32_t i = 0; i < mem1->num_dims; ++i)
    {
        if (mem1->shape[i] != mem2->shape[i]) return 0;
        if (mem1->stride[i] != mem2->stride[i]) return 0;
    }
    return 1;
}

int32_t sdp_mem_is_read_only(const sdp_Mem* mem)
{
    return (!mem || !mem->data) ? 1 : mem->is_read_only;
}

sdp_MemLocation sdp_mem_location(const sdp_Mem* mem)
{
    return mem ? mem->location : SDP_MEM_CPU;
}

int32_t sdp_mem_num_dims(const sdp_Mem* mem)
{
    return (!mem || !mem->data) ? 0 : mem->num_dims;
}

int64_t sdp_mem_num_elements(const sdp_Mem* mem)
{
    return (!mem || !mem->data) ? 0 : mem->num_elements;
}

void sdp_mem_random_fill(sdp_Mem* mem, sdp_Error* status)
{
    if (*status) return;
    if (mem->location != SDP_MEM_CPU)
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("Unsupported memory location");
        return;
    }
    int64_t n = mem->num_elements * (sdp_mem_is_complex(mem) ? 2 : 1);
    const int precision = mem->type & 0x0F;
    if (precision == SDP_MEM_FLOAT)
    {
        float* d = (float*)mem->data;
        for (int64_t i = 0; i < n; ++i) d[i] = (float)rand() / (float)RAND_MAX;
    }
    else if (precision == SDP_MEM_DOUBLE)
    {
        double* d = (double*)mem->data;
        for (int64_t i = 0; i < n; ++i) d[i] = (double)rand() / RAND_MAX;
    }
}

void sdp_mem_ref_dec(sdp_Mem* mem)
{
    sdp_mem_free(mem);
}

sdp_Mem* sdp_mem_ref_inc(sdp_Mem* mem)
{
    if (!mem) return nullptr;
    mem->ref_count++;
    return mem;
}

void sdp_mem_scale_real(sdp_Mem* mem, double value, sdp_Error* status)
{
    if (*status) return;
    if (!sdp_mem_is_c_contiguous(mem))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Array must be C contiguous");
        return;
    }
    const int64_t n = mem->num_elements;
    if (mem->location == SDP_MEM_CPU)
    {
        switch (mem->type)
        {
        case SDP_MEM_FLOAT:
            for (int64_t i = 0; i < n; ++i) ((float*)mem->data)[i] *= value;
            break;
        case SDP_MEM_DOUBLE:
            for (int64_t i = 0; i < n; ++i) ((double*)mem->data)[i] *= value;
            break;
        case SDP_MEM_COMPLEX_FLOAT:
            for (int64_t i = 0; i < n; ++i)
                ((float*)mem->data)[2 * i] *= value;
            break;
        case SDP_MEM_COMPLEX_DOUBLE:
            for (int64_t i = 0; i < n; ++i)
                ((double*)mem->data)[2 * i] *= value;
            break;
        default:
            *status = SDP_ERR_DATA_TYPE;
            SDP_LOG_ERROR("Unsupported data type");
        }
        return;
    }
    const unsigned int blocks = sdp_hip::blocks_for(n, 256);
    switch (mem->type)
    {
    case SDP_MEM_FLOAT:
        k_scale_real<float><<<blocks, 256>>>((float*)mem->data, n, value);
        break;
    case SDP_MEM_DOUBLE:
        k_scale_real<double><<<blocks, 256>>>((double*)mem->data, n, value);
        break;
    case SDP_MEM_COMPLEX_FLOAT:
        k_scale_real_complex<float><<<blocks, 256>>>(
                (float*)mem->data, n, value);
        break;
    case SDP_MEM_COMPLEX_DOUBLE:
        k_scale_real_complex<double><<<blocks, 256>>>(
                (double*)mem->data, n, value);
        break;
    default:
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data type");
        return;
    }
    SDP_HIP_CHECK_LAUNCH(status);
}

void sdp_mem_set_read_only(sdp_Mem* mem, int32_t value)
{
    if (mem) mem->is_read_only = value;
}

void sdp_mem_set_value(sdp_Mem* mem, int value, sdp_Error* status)
{
    if (*status || !mem) return;
    if (mem->num_dims < 1 || mem->num_dims > 3)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Unsupported number of dimensions (%d)", mem->num_dims);
        return;
    }
    int64_t n[3] = {1, 1, 1}, s[3] = {0, 0, 0};
    for (int32_t i = 0; i < mem->num_dims; ++i)
    {
        n[3 - mem->num_dims + i] = mem->shape[i];
        s[3 - mem->num_dims + i] = mem->stride[i];
    }
    if (mem->location == SDP_MEM_CPU)
    {
        switch (mem->type)
        {
        case SDP_MEM_INT: set_value_cpu<int, 1>(mem, value, n, s); break;
        case SDP_MEM_FLOAT: set_value_cpu<float, 1>(mem, value, n, s); break;
        case SDP_MEM_DOUBLE: set_value_cpu<double, 1>(mem, value, n, s); break;
        case SDP_MEM_COMPLEX_FLOAT:
            set_value_cpu<float, 2>(mem, value, n, s); break;
        case SDP_MEM_COMPLEX_DOUBLE:
            set_value_cpu<double, 2>(mem, value, n, s); break;
        default:
            *status = SDP_ERR_DATA_TYPE;
            SDP_LOG_ERROR("Unsupported data type");
        }
        return;
    }
    const unsigned int blocks = sdp_hip::blocks_for(n[0] * n[1] * n[2], 256);
    char* base = (char*)mem->data;
    switch (mem->type)
    {
    case SDP_MEM_INT:
        k_set_value<int, 1><<<blocks, 256>>>(base, n[0], n[1], n[2], s[0],
                s[1], s[2], value);
        break;
    case SDP_MEM_FLOAT:
        k_set_value<float, 1><<<blocks, 256>>>(base, n[0], n[1], n[2], s[0],
                s[1], s[2], (float)value);
        break;
    case SDP_MEM_DOUBLE:
        k_set_value<double, 1><<<blocks, 256>>>(base, n[0], n[1], n[2], s[0],
                s[1], s[2], (double)value);
        break;
    case SDP_MEM_COMPLEX_FLOAT:
        k_set_value<float, 2><<<blocks, 256>>>(base, n[0], n[1], n[2], s[0],
                s[1], s[2], (float)value);
        break;
    case SDP_MEM_COMPLEX_DOUBLE:
        k_set_value<double, 2><<<blocks, 256>>>(base, n[0], n[1], n[2], s[0],
                s[1], s[2], (double)value);
        break;
    default:
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data type");
        return;
    }
    SDP_HIP_CHECK_LAUNCH(status);
}

int64_t sdp_mem_shape_dim(const sdp_Mem* mem, int32_t dim)
{
    return (!mem || dim < 0 || dim >= mem->num_dims) ? 0 : mem->shape[dim];
}

int64_t sdp_mem_stride_bytes_dim(const sdp_Mem* mem, int32_t dim)
{
    return (!mem || dim < 0 || dim >= mem->num_dims) ? 0 : mem->stride[dim];
}

int64_t sdp_mem_stride_elements_dim(const sdp_Mem* mem, int32_t dim)
{
    const int64_t esize = mem ? sdp_mem_type_size(mem->type) : 0;
    return esize ? sdp_mem_stride_bytes_dim(mem, dim) / esize : 0;
}

sdp_MemType sdp_mem_type(const sdp_Mem* mem)
{
    return mem ? mem->type : SDP_MEM_VOID;
}

// ---- checkers (sdp_mem.h:591-993) -------------------------------------

void sdp_mem_check_writeable_at(const sdp_Mem* mem, sdp_Error* status,
        const char* expr, const char* func, const char* file, int line)
{
    if (*status) return;
    if (sdp_mem_is_read_only(mem))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        sdp_log_message(SDP_LOG_LEVEL_ERROR, stderr, func, file, line,
                "%s: Expected '%s' not to be read-only", func, expr);
    }
}

void sdp_mem_check_c_contiguity_at(const sdp_Mem* mem, sdp_Error* status,
        const char* expr, const char* func, const char* file, int line)
{
    if (*status) return;
    if (!sdp_mem_is_c_contiguous(mem))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        sdp_log_message(SDP_LOG_LEVEL_ERROR, stderr, func, file, line,
                "%s: Expected '%s' to be C contiguous", func, expr);
    }
}

void sdp_mem_check_location_at(const sdp_Mem* mem,
        sdp_MemLocation expected_location, sdp_Error* status,
        const char* expr, const char* func, const char* file, int line)
{
    if (*status) return;
    if (sdp_mem_location(mem) != expected_location)
    {
        *status = SDP_ERR_MEM_LOCATION;
        sdp_log_message(SDP_LOG_LEVEL_ERROR, stderr, func, file, line,
                "%s: Expected '%s' to be in %s memory (found %s)", func, expr,
                sdp_mem_location_name(expected_location),
                sdp_mem_location_name(sdp_mem_location(mem)));
    }
}

void sdp_mem_check_num_dims_at(const sdp_Mem* mem, int64_t expected_num_dims,
        sdp_Error* status, const char* expr, const char* func,
        const char* file, int line)
{
    if (*status) return;
    if (sdp_mem_num_dims(mem) != expected_num_dims)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        sdp_log_message(SDP_LOG_LEVEL_ERROR, stderr, func, file, line,
                "%s: Expected '%s' to have %lld dimensions (found %d)", func,
                expr, (long long)expected_num_dims, sdp_mem_num_dims(mem));
    }
}

void sdp_mem_check_dim_size_at(const sdp_Mem* mem, int32_t dim, int64_t size,
        sdp_Error* status, const char* expr, const char* func,
        const char* file, int line)
{
    if (*status) return;
    if (dim >= sdp_mem_num_dims(mem) || sdp_mem_shape_dim(mem, dim) != size)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        sdp_log_message(SDP_LOG_LEVEL_ERROR, stderr, func, file, line,
                "%s: Expected dimension %d of '%s' to have size %lld", func,
                dim, expr, (long long)size);
    }
}

void sdp_mem_check_shape_at(const sdp_Mem* mem, int32_t expected_num_dims,
        const int64_t* expected_shape, sdp_Error* status, const char* expr,
        const char* func, const char* file, int line)
{
    if (*status) return;
    sdp_mem_check_num_dims_at(mem, expected_num_dims, status, expr, func,
            file, line);
    for (int32_t i = 0; i < expected_num_dims && !*status; ++i)
    {
        sdp_mem_check_dim_size_at(mem, i, expected_shape[i], status, expr,
                func, file, line);
    }
}

void sdp_mem_check_shape_dim_at(const sdp_Mem* mem, int32_t dim,
        const int64_t expected_shape, sdp_Error* status, const char* expr,
        const char* func, const char* file, int line)
{
    sdp_mem_check_dim_size_at(mem, dim, expected_shape, status, expr, func,
            file, line);
}

void sdp_mem_check_same_shape_at(sdp_Mem* mem, int32_t dim, sdp_Mem* mem2,
        int32_t dim2, sdp_Error* status, const char* func, const char* expr,
        const char* expr2, const char* file, int line)
{
    if (*status) return;
    if (sdp_mem_shape_dim(mem, dim) != sdp_mem_shape_dim(mem2, dim2))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        sdp_log_message(SDP_LOG_LEVEL_ERROR, stderr, func, file, line,
                "%s: Expected dimension %d of '%s' to match dimension %d of "
                "'%s'", func, dim, expr, dim2, expr2);
    }
}

void sdp_mem_check_type_at(const sdp_Mem* mem, sdp_MemType expected_type,
        sdp_Error* status, const char* expr, const char* func,
        const char* file, int line)
{
    if (*status) return;
    if (sdp_mem_type(mem) != expected_type)
    {
        *status = SDP_ERR_DATA_TYPE;
        sdp_log_message(SDP_LOG_LEVEL_ERROR, stderr, func, file, line,
                "%s: Expected '%s' to be of type %s (found %s)", func, expr,
                sdp_mem_type_name(expected_type),
                sdp_mem_type_name(sdp_mem_type(mem)));
    }
}

} // extern "C"
