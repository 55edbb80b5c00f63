// Wave-level helpers specific to CDNA4 (gfx950).
#ifndef SDP_AMD_WAVE_OPS_H_
#define SDP_AMD_WAVE_OPS_H_

#include <hip/hip_runtime.h>

namespace sdp_hip {

// x summed over the four 16-lane rows of the wave (lane bits 4 and 5), in
// every lane. gfx950's row-swap permutes (v_permlane16_swap_b32,
// v_permlane32_swap_b32) move the data through the VALU instead of the LDS
// crossbar that ds_bpermute (__shfl_xor) takes. Float addition being
// commutative, the result equals that of
//   x += __shfl_xor(x, 16); x += __shfl_xor(x, 32);
__device__ __forceinline__ float sum_rows16(float x)
{
    const unsigned u = __float_as_uint(x);
    const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const unsigned v = __float_as_uint(x);
    const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

} // namespace sdp_hip

#endif
