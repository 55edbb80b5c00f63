// sdp_pswf_* C ABI (include/ska-sdp-func/fourier_transforms/sdp_pswf.h):
// prolate spheroidal wave functions S_mm(c, x) for the gridders' kernels
// and grid corrections, replacing src/ska-sdp-func/fourier_transforms/
// sdp_pswf.cpp:570-795 of ska-sdp-func 1.2.2. The function values come
// from the independent eigen-solver of grid_data/wtower_math.cpp (host
// tables, as the reference computes them on the host); device copies are
// made on request.
#include <cmath>
#include <complex>
#include <cstdlib>

#include "ska-sdp-func/fourier_transforms/sdp_pswf.h"
#include "ska-sdp-func/utility/sdp_logging.h"
#include "../grid_data/wtower_math.h"

struct sdp_Pswf
{
    int m;
    double c;
    sdp_wt::Pswf* fn;
    sdp_Mem* values;
    sdp_Mem* values_gpu;
    sdp_Mem* coeff;
    sdp_Mem* coeff_gpu;
};

namespace {

// sdp_pswf.cpp:570-601: out[0] = 0, out[size / 2] = S(0), symmetric
// values S(2 i / size) about the centre; end_correction puts 1e-15 in
// element 0 of an even-sized table.
template<typename T>
void fill(const sdp_wt::Pswf& fn, T* out, int size, int end_correction)
{
    out[0] = T(0.0);
    out[size / 2] = T(fn(0.0));
    for (int i = 1; i < size / 2; ++i)
    {
        const T v = T(fn(2.0 * i / size));
        out[size / 2 + i] = v;
        out[size / 2 - i] = v;
    }
    if (end_correction && size % 2 == 0) out[0] = T(1e-15);
}

void fill_mem(const sdp_wt::Pswf& fn, sdp_Mem* out, int end_correction,
        sdp_Error* status)
{
    const int size = (int)sdp_mem_shape_dim(out, 0);
    if (size <= 0) return;
    void* p = sdp_mem_data(out);
    switch (sdp_mem_type(out))
    {
    case SDP_MEM_DOUBLE:
        fill(fn, (double*)p, size, end_correction);
        break;
    case SDP_MEM_FLOAT:
        fill(fn, (float*)p, size, end_correction);
        break;
    case SDP_MEM_COMPLEX_FLOAT:
        fill(fn, (std::complex<float>*)p, size, end_correction);
        break;
    case SDP_MEM_COMPLEX_DOUBLE:
        fill(fn, (std::complex<double>*)p, size, end_correction);
        break;
    default:
        *status = SDP_ERR_DATA_TYPE;
    }
}

} // namespace

extern "C" {

sdp_Pswf* sdp_pswf_create(int m, double c)
{
    sdp_Error status = SDP_SUCCESS;
    sdp_Pswf* plan = (sdp_Pswf*)calloc(1, sizeof(sdp_Pswf));
    plan->m = m;
    plan->c = c;
    plan->fn = new sdp_wt::Pswf(sdp_wt::make_pswf_order(c, m));
    const int64_t n = (int64_t)plan->fn->coef.size();
    plan->coeff = sdp_mem_create(SDP_MEM_DOUBLE, SDP_MEM_CPU, 1, &n, &status);
    if (!status)
    {
        double* d = (double*)sdp_mem_data(plan->coeff);
        for (int64_t k = 0; k < n; ++k) d[k] = plan->fn->coef[k];
    }
    return plan;
}

const sdp_Mem* sdp_pswf_coeff(sdp_Pswf* plan, sdp_MemLocation location,
        sdp_Error* status)
{
    if (!plan) return nullptr;
    if (location == SDP_MEM_GPU)
    {
        if (!plan->coeff_gpu)
            plan->coeff_gpu = sdp_mem_create_copy(plan->coeff, location,
                    status);
        return plan->coeff_gpu;
    }
    return plan->coeff;
}

const sdp_Mem* sdp_pswf_values(sdp_Pswf* plan, sdp_MemLocation location,
        sdp_Error* status)
{
    if (!plan) return nullptr;
    if (location == SDP_MEM_GPU && plan->values)
    {
        if (!plan->values_gpu)
            plan->values_gpu = sdp_mem_create_copy(plan->values, location,
                    status);
        return plan->values_gpu;
    }
    return plan->values;
}

double sdp_pswf_evaluate(const sdp_Pswf* plan, double x)
{
    const double ax = std::fabs(x);
    return ax < 1.0 ? (*plan->fn)(ax) : 0.0;
}

double sdp_pswf_par_c(const sdp_Pswf* plan)
{
    return plan->c;
}

double sdp_pswf_par_m(const sdp_Pswf* plan)
{
    return plan->m;
}

void sdp_pswf_free(sdp_Pswf* plan)
{
    if (!plan) return;
    sdp_mem_free(plan->values);
    sdp_mem_free(plan->values_gpu);
    sdp_mem_free(plan->coeff);
    sdp_mem_free(plan->coeff_gpu);
    delete plan->fn;
    free(plan);
}

void sdp_pswf_generate(sdp_Pswf* plan, sdp_Mem* out, int size,
        int end_correction, sdp_Error* status)
{
    if (*status) return;
    sdp_Mem* dst = out;
    if (out && size == 0)
    {
        if (sdp_mem_num_dims(out) != 1)
        {
            *status = SDP_ERR_INVALID_ARGUMENT;
            return;
        }
        if (sdp_mem_location(out) != SDP_MEM_CPU)
        {
            *status = SDP_ERR_MEM_LOCATION;
            return;
        }
    }
    else if (!out && size > 0)
    {
        sdp_mem_free(plan->values);
        sdp_mem_free(plan->values_gpu);
        plan->values_gpu = nullptr;
        const int64_t shape[] = {size};
        plan->values = sdp_mem_create(SDP_MEM_DOUBLE, SDP_MEM_CPU, 1, shape,
                status);
        dst = plan->values;
    }
    else
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Must specify only one of 'out' or 'size'");
        return;
    }
    if (*status) return;
    fill_mem(*plan->fn, dst, end_correction, status);
}

void sdp_generate_pswf(int m, double c, sdp_Mem* out, sdp_Error* status)
{
    if (*status) return;
    sdp_Pswf* plan = sdp_pswf_create(m, c);
    sdp_pswf_generate(plan, out, 0, 0, status);
    sdp_pswf_free(plan);
}

} // extern "C"
