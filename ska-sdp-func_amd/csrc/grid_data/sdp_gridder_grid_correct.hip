// Image-plane grid correction of the w-towers path: the drop-in C ABI of
// include/ska-sdp-func/grid_data/sdp_gridder_grid_correct.h, replacing
// src/ska-sdp-func/grid_data/sdp_gridder_grid_correct.cpp:18-326 and its
// kernels (sdp_gridder_grid_correct.cu:15, :54) of ska-sdp-func 1.2.2.
//
// One thread per facet pixel; the per-pixel arithmetic is the w-towers
// plan's (wtower_plan.h: PSWF table lookups for l and m, the Legendre
// series of pswf_n at |2 w_step n|, the product inverted in double and
// applied in the facet's precision; the w-stacking phasor from a reduced
// phase). Host facets are staged through device memory.
#include <algorithm>
#include <cmath>
#include <vector>

#include "ska-sdp-func/grid_data/sdp_gridder_grid_correct.h"
#include "wtower_math.h"
#include "wtower_ops.h"
#include "wtower_plan.h"
#include "../utility/sdp_hip.h"

using namespace sdp_wt;

namespace {

// mode 0: PSWF correction (pixels outside the image unchanged);
// mode 1: w-stacking phasor only (every pixel, scale 1 exactly).
__global__ void k_correct(AnyView facet, int nl, int nm, int off_l,
        int off_m, CorrParams cp, int mode)
{
    const int im = blockIdx.x * blockDim.x + threadIdx.x;
    if (im >= nm) return;
    // Rows stride over the y-grid (capped at 65535 blocks by the host).
    for (int il = blockIdx.y; il < nl; il += gridDim.y)
    {
        const int pl = il - nl / 2 + off_l, pm = im - nm / 2 + off_m;
        const int64_t i = (int64_t)il * nm + im;
        if (mode == 0)
        {
            if (!corr_inside(pl, pm, cp)) continue;
            facet.store(i, correct_scaled(facet.load(i), facet.kind, pl, pm,
                    cp, pixel_scale(pl, pm, cp)));
        }
        else
        {
            facet.store(i, correct_scaled(facet.load(i), facet.kind, pl, pm,
                    cp, 1.0));
        }
    }
}

struct DevTable
{
    double* ptr = nullptr;

    void upload(const std::vector<double>& h, sdp_Error* status)
    {
        if (*status || h.empty()) return;
        SDP_HIP_CHECK(hipMalloc((void**)&ptr, h.size() * sizeof(double)),
                status);
        if (*status) return;
        SDP_HIP_CHECK(hipMemcpy(ptr, h.data(), h.size() * sizeof(double),
                hipMemcpyHostToDevice), status);
    }

    ~DevTable()
    {
        if (ptr) (void)hipFree(ptr);   // hipFree waits for the kernel
    }
};

bool check_facet(const sdp_Mem* facet, bool complex_only, sdp_Error* status)
{
    if (*status) return false;
    const int kind = any_kind(sdp_mem_type(facet));
    if (kind < 0 || (complex_only && kind < 2))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported facet data type");
        return false;
    }
    if (sdp_mem_num_dims(facet) != 2 || !sdp_mem_is_c_contiguous(facet))
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Facet must be a 2-D C-contiguous array");
        return false;
    }
    const sdp_MemLocation loc = sdp_mem_location(facet);
    if (loc != SDP_MEM_CPU && loc != SDP_MEM_GPU)
    {
        *status = SDP_ERR_MEM_LOCATION;
        return false;
    }
    if (!sdp_hip::device_available())
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("No GPU available for the grid correction");
        return false;
    }
    return true;
}

void launch(sdp_Mem* facet, int off_l, int off_m, const CorrParams& cp,
        int mode, sdp_Error* status)
{
    Staged f;
    f.init(facet, status);
    if (*status) return;
    const int nl = (int)sdp_mem_shape_dim(facet, 0);
    const int nm = (int)sdp_mem_shape_dim(facet, 1);
    if (nl <= 0 || nm <= 0) return;
    const AnyView v = {sdp_mem_data(f.dev), any_kind(sdp_mem_type(facet))};
    k_correct<<<dim3((nm + 255) / 256, std::min(nl, 65535)), 256>>>(v, nl,
            nm, off_l, off_m,
            cp, mode);
    SDP_HIP_CHECK_LAUNCH(status);
    f.write_back(status);
}

CorrParams base_params(int image_size, double theta, double w_step,
        double shear_u, double shear_v)
{
    CorrParams cp{};
    cp.image_size = image_size;
    cp.theta = theta;
    cp.w_step = w_step;
    cp.shear_u = shear_u;
    cp.shear_v = shear_v;
    return cp;
}

} // namespace

extern "C" {

void sdp_gridder_grid_correct_pswf(int image_size, double theta,
        double w_step, double shear_u, double shear_v, int support,
        int w_support, sdp_Mem* facet, int facet_offset_l,
        int facet_offset_m, sdp_Error* status)
{
    if (!check_facet(facet, false, status)) return;
    if (image_size <= 0)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        return;
    }
    // sdp_gridder_grid_correct.cpp:134-136: pswf of c = support pi / 2 on
    // image_size points (end-corrected), pswf_n of c = w_support pi / 2.
    DevTable lm, pn;
    lm.upload(generate_pswf(support * (M_PI / 2), image_size, true), status);
    const Pswf fn = make_pswf(w_support * (M_PI / 2));
    pn.upload(fn.coef, status);
    if (*status) return;
    CorrParams cp = base_params(image_size, theta, w_step, shear_u, shear_v);
    cp.pswf_lm = lm.ptr;
    cp.pswf_n = pn.ptr;
    cp.n_pswf_n = (int)fn.coef.size();
    cp.c_n = w_support * (M_PI / 2);
    cp.w_offset = 0;
    launch(facet, facet_offset_l, facet_offset_m, cp, 0, status);
}

void sdp_gridder_grid_correct_w_stack(int image_size, double theta,
        double w_step, double shear_u, double shear_v, sdp_Mem* facet,
        int facet_offset_l, int facet_offset_m, int w_offset, int inverse,
        sdp_Error* status)
{
    if (*status || w_offset == 0) return;
    if (!check_facet(facet, true, status)) return;
    CorrParams cp = base_params(image_size, theta, w_step, shear_u, shear_v);
    cp.w_offset = w_offset;
    cp.inverse = inverse ? 1 : 0;
    launch(facet, facet_offset_l, facet_offset_m, cp, 1, status);
}

} // extern "C"
