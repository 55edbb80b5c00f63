/* MI355X-native ska-sdp-func hot path: error codes.
 *
 * Drop-in for the reference enum at
 *   src/ska-sdp-func/utility/sdp_errors.h:13-37
 * Same numeric values (0..6); the Python wrapper maps them to
 * "Error N: <meaning>" strings exactly as the reference's
 * src/ska_sdp_func/utility/error_checking.py:11-19 does.
 */
#ifndef SDP_ERRORS_H_
#define SDP_ERRORS_H_

#ifdef __cplusplus
extern "C" {
#endif

enum sdp_Error
{
    SDP_SUCCESS = 0,
    SDP_ERR_RUNTIME = 1,
    SDP_ERR_INVALID_ARGUMENT = 2,
    SDP_ERR_DATA_TYPE = 3,
    SDP_ERR_MEM_ALLOC_FAILURE = 4,
    SDP_ERR_MEM_COPY_FAILURE = 5,
    SDP_ERR_MEM_LOCATION = 6
};
typedef enum sdp_Error sdp_Error;

#ifdef __cplusplus
}
#endif

#endif
