// SKA-format logging (drop-in for src/ska-sdp-func/utility/sdp_logging.c).
// Format "1|<utc>|LEVEL||func|file#line|| msg"; filter from the environment
// variable SKA_SDP_FUNC_LOG_LEVEL (debug/info/warn/err/crit, default info).
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>
#include <sys/time.h>

#include "ska-sdp-func/utility/sdp_logging.h"

namespace {

sdp_LogLevel filter_from_env()
{
    const char* env = std::getenv("SKA_SDP_FUNC_LOG_LEVEL");
    if (!env) return SDP_LOG_LEVEL_INFO;
    struct { const char* key; sdp_LogLevel level; } table[] = {
        {"debug", SDP_LOG_LEVEL_DEBUG}, {"info", SDP_LOG_LEVEL_INFO},
        {"warn", SDP_LOG_LEVEL_WARNING}, {"err", SDP_LOG_LEVEL_ERROR},
        {"crit", SDP_LOG_LEVEL_CRITICAL}
    };
    for (const auto& t : table)
    {
        if (!strncasecmp(env, t.key, strlen(t.key))) return t.level;
    }
    return SDP_LOG_LEVEL_UNDEF;   // unknown value: log everything
}

const char* level_name(sdp_LogLevel level)
{
    switch (level)
    {
    case SDP_LOG_LEVEL_DEBUG: return "DEBUG";
    case SDP_LOG_LEVEL_INFO: return "INFO";
    case SDP_LOG_LEVEL_WARNING: return "WARNING";
    case SDP_LOG_LEVEL_ERROR: return "ERROR";
    case SDP_LOG_LEVEL_CRITICAL: return "CRITICAL";
    default: return "UNDEF";
    }
}

} // namespace

extern "C" void sdp_log_message(sdp_LogLevel level, FILE* stream,
        const char* func, const char* file, int line, const char* message, ...)
{
    static const sdp_LogLevel filter = filter_from_env();
    if (level < filter) return;
    static std::mutex mutex;
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    struct tm t;
    gmtime_r(&tv.tv_sec, &t);
    char stamp[48];
    snprintf(stamp, sizeof(stamp), "%04d-%02d-%02dT%02d:%02d:%02d.%03dZ",
            t.tm_year + 1900, t.tm_mon + 1, t.tm_mday, t.tm_hour, t.tm_min,
            t.tm_sec, (int)(tv.tv_usec / 1000));
    const char* base = file ? strrchr(file, '/') : nullptr;
    std::lock_guard<std::mutex> lock(mutex);
    fprintf(stream, "1|%s|%s||%s|%s#%d|| ", stamp, level_name(level), func,
            base ? base + 1 : (file ? file : ""), line);
    va_list args;
    va_start(args, message);
    vfprintf(stream, message, args);
    va_end(args);
    fputc('\n', stream);
    fflush(stream);
}
