// Element-wise sub-grid operations of the w-towers path (device), shared by
// the gridder (sdp_gridder_wtower_uvw.hip) and the utility C ABI
// (sdp_gridder_utils.hip), plus host staging of CPU arrays.
#ifndef SDP_WTOWER_OPS_H_
#define SDP_WTOWER_OPS_H_

#include <cstdint>

#include "ska-sdp-func/utility/sdp_mem.h"
#include "wtower_dev.h"

namespace sdp_wt {

// out = in1 / w_pattern ** exponent, computed in complex double
// (sdp_gridder_utils.cu:132-150); n elements, stream 0.
void wt_scale_inv(AnyView out, AnyView in1, const double* w_pattern,
        int exponent, int64_t n, sdp_Error* status);

// out += in1 * w_pattern ** exponent (w_pattern may be null: out += in1;
// a real out takes in1's real part and ignores the pattern, as
// sdp_gridder_utils.cu:16-52).
void wt_accum(AnyView out, AnyView in1, const double* w_pattern,
        int exponent, int64_t n, sdp_Error* status);

// data *= (-1)^(i + j) for an nx x ny complex array (sdp_fft_phase).
template<typename T>
void wt_fft_phase(T* data, int nx, int ny, sdp_Error* status);

// Bounds of the scaled (u, v, w) of the selected channels of device arrays
// (sdp_gridder_uvw_bounds_all, utils.cpp:682-719): +inf / -inf when no
// channel is selected. Synchronises with the device.
template<typename U>
void uvw_bounds_dev(const U* uvws, int64_t rows, double f0, double df,
        const int* start_chs, const int* end_chs, double lo[3], double hi[3],
        sdp_Error* status);

// Device view of an sdp_Mem: the array itself when on the GPU, otherwise a
// staged device copy (written back by write_back()).
struct Staged
{
    sdp_Mem* dev = nullptr;
    const sdp_Mem* src = nullptr;
    bool copy = false;

    void init(const sdp_Mem* m, sdp_Error* status);
    void write_back(sdp_Error* status);
    ~Staged();
};

} // namespace sdp_wt

#endif
