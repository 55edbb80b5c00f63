/* Small maths macros of the drop-in C ABI.
 *
 * Same names and meaning as src/ska-sdp-func/math/sdp_math_macros.h
 * (ska-sdp-func 1.2.2), which the reference's sdp_gridder_clamp_channels.h
 * and sdp_gridder_utils.h include: SDP_INLINE, M_PI, C_0 (speed of light,
 * m/s), MAX, MIN. SDP_INLINE is `static inline` here so that header-only
 * functions compile as C99 and as C++ without an external definition. The
 * library's device code does not use these (it has its own __device__
 * helpers); they are for C / C++ callers of the headers.
 */
#ifndef SDP_MATH_MACROS_H_
#define SDP_MATH_MACROS_H_

#ifdef __cplusplus
#include <cmath>
#else
#include <math.h>
#endif

#ifndef SDP_INLINE
#define SDP_INLINE static inline
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846264338327950288
#endif

/* Speed of light in vacuum, m/s. */
#define C_0 299792458.0

#define MAX(X, Y) ((X) > (Y) ? (X) : (Y))
#define MIN(X, Y) ((X) < (Y) ? (X) : (Y))

#endif /* SDP_MATH_MACROS_H_ */
