/* MI355X-native ska-sdp-func hot path: the sdp_Mem tensor handle.
 *
 * Drop-in C ABI for src/ska-sdp-func/utility/sdp_mem.h of the reference
 * (declarations at sdp_mem.h:140-993; implementation sdp_mem.cpp). The
 * Python ctypes wrapper binds sdp_mem_create_wrapper / sdp_mem_set_read_only /
 * sdp_mem_free exactly as src/ska_sdp_func/utility/mem.py:124-136 does.
 *
 * Semantics kept from the reference:
 *  - byte strides (Python/numpy compatible), computed from the shape if NULL;
 *  - a wrapper never owns its data; sdp_mem_create allocates and owns it
 *    (host: calloc; GPU: hipMalloc on the current HIP device);
 *  - reference counting through sdp_mem_ref_inc / sdp_mem_free;
 *  - sdp_mem_gpu_buffer[_const] returns a POINTER TO the data pointer (so it
 *    can be dropped into a kernel-argument array) and fails with
 *    SDP_ERR_MEM_LOCATION for host memory.
 */
#ifndef SDP_MEM_H_
#define SDP_MEM_H_

#include <stdint.h>

#include "ska-sdp-func/utility/sdp_errors.h"
#include "ska-sdp-func/utility/sdp_logging.h"

#ifdef __cplusplus
extern "C" {
#endif

struct sdp_Mem;
typedef struct sdp_Mem sdp_Mem;

/* Opaque stream handle (reference: utility/sdp_device_wrapper.h:28-33).
 * Here it wraps a hipStream_t. */
struct sdp_CudaStream;
typedef struct sdp_CudaStream sdp_CudaStream;

enum sdp_MemType
{
    SDP_MEM_VOID = 0,
    SDP_MEM_CHAR = 1,
    SDP_MEM_INT = 2,
    SDP_MEM_FLOAT = 4,
    SDP_MEM_DOUBLE = 8,
    SDP_MEM_COMPLEX = 32,
    SDP_MEM_COMPLEX_FLOAT = SDP_MEM_FLOAT | SDP_MEM_COMPLEX,
    SDP_MEM_COMPLEX_DOUBLE = SDP_MEM_DOUBLE | SDP_MEM_COMPLEX
};
typedef enum sdp_MemType sdp_MemType;

enum sdp_MemLocation
{
    SDP_MEM_CPU,
    SDP_MEM_GPU
};
typedef enum sdp_MemLocation sdp_MemLocation;

/* sdp_mem.h:140 */
sdp_Mem* sdp_mem_create(sdp_MemType type, sdp_MemLocation location,
        int32_t num_dims, const int64_t* shape, sdp_Error* status);

/* sdp_mem.h:168 (Python: mem.py:124-136) */
sdp_Mem* sdp_mem_create_wrapper(void* data, sdp_MemType type,
        sdp_MemLocation location, int32_t num_dims, const int64_t* shape,
        const int64_t* stride, sdp_Error* status);

/* sdp_mem.h:193 */
sdp_Mem* sdp_mem_create_wrapper_for_slice(const sdp_Mem* src,
        const int64_t* slice_offsets, const int32_t num_dims_slice,
        const int64_t* slice_shape, sdp_Error* status);

/* sdp_mem.h:207 */
sdp_Mem* sdp_mem_create_alias(const sdp_Mem* src);

/* sdp_mem.h:217 */
sdp_Mem* sdp_mem_create_copy(const sdp_Mem* src, sdp_MemLocation location,
        sdp_Error* status);

/* sdp_mem.h:229 */
void sdp_mem_clear_contents(sdp_Mem* mem, sdp_Error* status);

/* sdp_mem.h:239 */
void sdp_mem_clear_portion(sdp_Mem* mem, int64_t start_index,
        int64_t num_elements, sdp_Error* status);

/* sdp_mem.h:255 */
sdp_Mem* sdp_mem_convert_precision(const sdp_Mem* src,
        sdp_MemType output_type, sdp_Error* status);

/* sdp_mem.h:271 */
void sdp_mem_copy_contents(sdp_Mem* dst, const sdp_Mem* src,
        int64_t offset_dst, int64_t offset_src, int64_t num_elements,
        sdp_Error* status);

/* sdp_mem.h:293 */
void sdp_mem_copy_contents_async(sdp_Mem* dst, const sdp_Mem* src,
        int64_t offset_dst, int64_t offset_src, int64_t num_elements,
        sdp_CudaStream* stream, sdp_Error* status);

/* sdp_mem.h:309-345 */
void* sdp_mem_data(sdp_Mem* mem);
const void* sdp_mem_data_const(const sdp_Mem* mem);
void* sdp_mem_gpu_buffer(sdp_Mem* mem, sdp_Error* status);
const void* sdp_mem_gpu_buffer_const(const sdp_Mem* mem, sdp_Error* status);

/* sdp_mem.h:357-575 */
void sdp_mem_free(sdp_Mem* mem);
int32_t sdp_mem_is_c_contiguous(const sdp_Mem* mem);
int32_t sdp_mem_is_floating_point(const sdp_Mem* mem);
int32_t sdp_mem_is_complex(const sdp_Mem* mem);
int32_t sdp_mem_is_complex4(const sdp_Mem* mem);
int32_t sdp_mem_is_double(const sdp_Mem* mem);
int32_t sdp_mem_is_matching(const sdp_Mem* mem1, const sdp_Mem* mem2,
        int32_t check_location);
int32_t sdp_mem_is_read_only(const sdp_Mem* mem);
sdp_MemLocation sdp_mem_location(const sdp_Mem* mem);
int32_t sdp_mem_num_dims(const sdp_Mem* mem);
int64_t sdp_mem_num_elements(const sdp_Mem* mem);
void sdp_mem_random_fill(sdp_Mem* mem, sdp_Error* status);
void sdp_mem_ref_dec(sdp_Mem* mem);
sdp_Mem* sdp_mem_ref_inc(sdp_Mem* mem);
void sdp_mem_scale_real(sdp_Mem* mem, double value, sdp_Error* status);
void sdp_mem_set_read_only(sdp_Mem* mem, int32_t value);
void sdp_mem_set_value(sdp_Mem* mem, int value, sdp_Error* status);
int64_t sdp_mem_shape_dim(const sdp_Mem* mem, int32_t dim);
int64_t sdp_mem_stride_bytes_dim(const sdp_Mem* mem, int32_t dim);
int64_t sdp_mem_stride_elements_dim(const sdp_Mem* mem, int32_t dim);
sdp_MemType sdp_mem_type(const sdp_Mem* mem);
int64_t sdp_mem_type_size(sdp_MemType type);
const char* sdp_mem_location_name(sdp_MemLocation location);
const char* sdp_mem_type_name(sdp_MemType type);

/* Checkers: sdp_mem.h:591-993. Each sets *status and logs on failure. */
void sdp_mem_check_writeable_at(const sdp_Mem* mem, sdp_Error* status,
        const char* expr, const char* func, const char* file, int line);
void sdp_mem_check_c_contiguity_at(const sdp_Mem* mem, sdp_Error* status,
        const char* expr, const char* func, const char* file, int line);
void sdp_mem_check_location_at(const sdp_Mem* mem,
        sdp_MemLocation expected_location, sdp_Error* status,
        const char* expr, const char* func, const char* file, int line);
void sdp_mem_check_num_dims_at(const sdp_Mem* mem, int64_t expected_num_dims,
        sdp_Error* status, const char* expr, const char* func,
        const char* file, int line);
void sdp_mem_check_dim_size_at(const sdp_Mem* mem, int32_t dim, int64_t size,
        sdp_Error* status, const char* expr, const char* func,
        const char* file, int line);
void sdp_mem_check_shape_at(const sdp_Mem* mem, int32_t expected_num_dims,
        const int64_t* expected_shape, sdp_Error* status, const char* expr,
        const char* func, const char* file, int line);
void sdp_mem_check_shape_dim_at(const sdp_Mem* mem, int32_t dim,
        const int64_t expected_shape, sdp_Error* status, const char* expr,
        const char* func, const char* file, int line);
void sdp_mem_check_same_shape_at(sdp_Mem* mem, int32_t dim, sdp_Mem* mem2,
        int32_t dim2, sdp_Error* status, const char* func, const char* expr,
        const char* expr2, const char* file, int line);
void sdp_mem_check_type_at(const sdp_Mem* mem, sdp_MemType expected_type,
        sdp_Error* status, const char* expr, const char* func,
        const char* file, int line);

#define sdp_mem_check_writeable(mem, status) sdp_mem_check_writeable_at( \
        mem, status, #mem, __func__, FILENAME, __LINE__)
#define sdp_mem_check_c_contiguity(mem, status) \
    sdp_mem_check_c_contiguity_at(mem, status, #mem, __func__, FILENAME, \
        __LINE__)
#define sdp_mem_check_location(mem, loc, status) sdp_mem_check_location_at( \
        mem, loc, status, #mem, __func__, FILENAME, __LINE__)
#define sdp_mem_check_num_dims(mem, n, status) sdp_mem_check_num_dims_at( \
        mem, n, status, #mem, __func__, FILENAME, __LINE__)
#define sdp_mem_check_dim_size(mem, dim, size, status) \
    sdp_mem_check_dim_size_at(mem, dim, size, status, #mem, __func__, \
        FILENAME, __LINE__)
#define sdp_mem_check_shape(mem, n, shape, status) sdp_mem_check_shape_at( \
        mem, n, shape, status, #mem, __func__, FILENAME, __LINE__)
#define sdp_mem_check_shape_dim(mem, dim, size, status) \
    sdp_mem_check_shape_dim_at(mem, dim, size, status, #mem, __func__, \
        FILENAME, __LINE__)
#define sdp_mem_check_same_shape(mem, dim, mem2, dim2, status) \
    sdp_mem_check_same_shape_at(mem, dim, mem2, dim2, status, __func__, \
        #mem, #mem2, __FILE__, __LINE__)
#define sdp_mem_check_type(mem, type, status) sdp_mem_check_type_at( \
        mem, type, status, #mem, __func__, FILENAME, __LINE__)

#ifdef __cplusplus
}
#endif

#endif
