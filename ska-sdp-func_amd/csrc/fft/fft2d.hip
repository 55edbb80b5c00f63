// rocFFT-backed 2-D C2C transform (see fft2d.h).
#include <mutex>

#include <rocfft/rocfft.h>

#include "fft2d.h"
#include "../utility/sdp_hip.h"

namespace sdp_fft {

struct Plan2D
{
    rocfft_plan forward = nullptr;
    rocfft_plan inverse = nullptr;
    rocfft_execution_info info = nullptr;
    void* work = nullptr;
    size_t work_bytes = 0;
};

namespace {

bool setup(sdp_Error* status)
{
    static std::once_flag once;
    static rocfft_status result = rocfft_status_success;
    std::call_once(once, [] { result = rocfft_setup(); });
    if (result != rocfft_status_success)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("rocfft_setup failed (%d)", (int)result);
        return false;
    }
    return true;
}

} // namespace

Plan2D* create_2d(int n_slow, int n_fast, bool dbl, sdp_Error* status)
{
    return create_2d_batched(n_slow, n_fast, dbl, 1,
            (size_t)n_slow * n_fast, status);
}

Plan2D* create_2d_batched(int n_slow, int n_fast, bool dbl, size_t batch,
        size_t distance, sdp_Error* status)
{
    if (*status) return nullptr;
    if (!sdp_hip::device_available())
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("No HIP device available for the FFT");
        return nullptr;
    }
    if (!setup(status)) return nullptr;
    Plan2D* p = new Plan2D;
    const size_t lengths[2] = {(size_t)n_fast, (size_t)n_slow};
    const rocfft_precision prec =
            dbl ? rocfft_precision_double : rocfft_precision_single;
    rocfft_plan_description desc = nullptr;
    if (batch > 1 || distance != (size_t)n_slow * n_fast)
    {
        const size_t strides[2] = {1, (size_t)n_fast};
        rocfft_plan_description_create(&desc);
        rocfft_plan_description_set_data_layout(desc,
                rocfft_array_type_complex_interleaved,
                rocfft_array_type_complex_interleaved, nullptr, nullptr,
                2, strides, distance, 2, strides, distance);
    }
    rocfft_status e1 = rocfft_plan_create(&p->forward,
            rocfft_placement_inplace, rocfft_transform_type_complex_forward,
            prec, 2, lengths, batch, desc);
    rocfft_status e2 = rocfft_plan_create(&p->inverse,
            rocfft_placement_inplace, rocfft_transform_type_complex_inverse,
            prec, 2, lengths, batch, desc);
    if (desc) rocfft_plan_description_destroy(desc);
    if (e1 != rocfft_status_success || e2 != rocfft_status_success)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("rocfft_plan_create failed (%d, %d)", (int)e1, (int)e2);
        destroy_2d(p);
        return nullptr;
    }
    size_t w1 = 0, w2 = 0;
    rocfft_plan_get_work_buffer_size(p->forward, &w1);
    rocfft_plan_get_work_buffer_size(p->inverse, &w2);
    p->work_bytes = w1 > w2 ? w1 : w2;
    rocfft_execution_info_create(&p->info);
    if (p->work_bytes)
    {
        SDP_HIP_CHECK(hipMalloc(&p->work, p->work_bytes), status);
        if (*status)
        {
            destroy_2d(p);
            return nullptr;
        }
        rocfft_execution_info_set_work_buffer(p->info, p->work, p->work_bytes);
    }
    return p;
}

void exec_2d(Plan2D* plan, void* data, bool forward, hipStream_t stream,
        sdp_Error* status)
{
    if (*status || !plan) return;
    rocfft_execution_info_set_stream(plan->info, stream);
    void* buffers[1] = {data};
    const rocfft_status e = rocfft_execute(
            forward ? plan->forward : plan->inverse, buffers, nullptr,
            plan->info);
    if (e != rocfft_status_success)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("rocfft_execute failed (%d)", (int)e);
    }
}

void destroy_2d(Plan2D* plan)
{
    if (!plan) return;
    if (plan->forward) rocfft_plan_destroy(plan->forward);
    if (plan->inverse) rocfft_plan_destroy(plan->inverse);
    if (plan->info) rocfft_execution_info_destroy(plan->info);
    if (plan->work) (void)hipFree(plan->work);
    delete plan;
}

} // namespace sdp_fft
