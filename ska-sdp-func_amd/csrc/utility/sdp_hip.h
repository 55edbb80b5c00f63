// Internal HIP helpers for the MI355X-native ska-sdp-func hot path.
#ifndef SDP_HIP_INTERNAL_H_
#define SDP_HIP_INTERNAL_H_

#include <hip/hip_runtime.h>

#include "ska-sdp-func/utility/sdp_errors.h"
#include "ska-sdp-func/utility/sdp_logging.h"

// Sets *status = SDP_ERR_RUNTIME and logs if a HIP call fails.
#define SDP_HIP_CHECK(call, status) \
    do { \
        const hipError_t sdp_hip_err_ = (call); \
        if (sdp_hip_err_ != hipSuccess) { \
            if (!*(status)) *(status) = SDP_ERR_RUNTIME; \
            SDP_LOG_ERROR("HIP error %d (%s) in %s", (int)sdp_hip_err_, \
                    hipGetErrorString(sdp_hip_err_), #call); \
        } \
    } while (0)

// Checks the last kernel launch.
#define SDP_HIP_CHECK_LAUNCH(status) SDP_HIP_CHECK(hipGetLastError(), status)

namespace sdp_hip {

// True if at least one HIP device is visible (cached after first query).
bool device_available();

// Grid sizing helper.
inline unsigned int blocks_for(long long n, int threads)
{
    return (unsigned int)((n + threads - 1) / threads);
}

} // namespace sdp_hip

#endif
