/* MI355X-native ska-sdp-func hot path: SKA-format logging.
 *
 * Replaces src/ska-sdp-func/utility/sdp_logging.h:27-95 (macros and
 * sdp_log_message). Output format "1|<utc>|LEVEL||func|file#line|| msg",
 * filtered by the SKA_SDP_FUNC_LOG_LEVEL environment variable
 * (reference: sdp_logging.c:28-54, 108).
 */
#ifndef SDP_LOGGING_H_
#define SDP_LOGGING_H_

#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

enum sdp_LogLevel
{
    SDP_LOG_LEVEL_UNDEF,
    SDP_LOG_LEVEL_DEBUG,
    SDP_LOG_LEVEL_INFO,
    SDP_LOG_LEVEL_WARNING,
    SDP_LOG_LEVEL_ERROR,
    SDP_LOG_LEVEL_CRITICAL
};
typedef enum sdp_LogLevel sdp_LogLevel;

void sdp_log_message(
        sdp_LogLevel level,
        FILE* stream,
        const char* func,
        const char* file,
        int line,
        const char* message,
        ...
);

#ifdef __cplusplus
}
#endif

#ifndef FILENAME
#define FILENAME __FILE__
#endif

#define SDP_LOG_CRITICAL(...) sdp_log_message(SDP_LOG_LEVEL_CRITICAL, \
        stderr, __func__, FILENAME, __LINE__, __VA_ARGS__)
#define SDP_LOG_ERROR(...) sdp_log_message(SDP_LOG_LEVEL_ERROR, \
        stderr, __func__, FILENAME, __LINE__, __VA_ARGS__)
#define SDP_LOG_WARNING(...) sdp_log_message(SDP_LOG_LEVEL_WARNING, \
        stderr, __func__, FILENAME, __LINE__, __VA_ARGS__)
#define SDP_LOG_INFO(...) sdp_log_message(SDP_LOG_LEVEL_INFO, \
        stdout, __func__, FILENAME, __LINE__, __VA_ARGS__)
#define SDP_LOG_DEBUG(...) sdp_log_message(SDP_LOG_LEVEL_DEBUG, \
        stdout, __func__, FILENAME, __LINE__, __VA_ARGS__)

#endif
