// log.cpp -- see log.h
#include "log.h"

#include <cstdio>
#include <mutex>

namespace bcm3 {

static LogLevel g_level = LogLevel::Warning;
static std::mutex g_mutex;
static thread_local std::string g_last_error;

void log_set_level(LogLevel l) { g_level = l; }

void log_message(LogLevel level, const char* fmt, ...)
{
    char buf[2048];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (level == LogLevel::Error) g_last_error = buf;
    if (level < g_level) return;
    std::lock_guard<std::mutex> lock(g_mutex);
    fprintf(level == LogLevel::Info ? stdout : stderr, "%s%s\n",
            level == LogLevel::Error ? "ERROR: " : (level == LogLevel::Warning ? "WARNING: " : ""), buf);
    fflush(level == LogLevel::Info ? stdout : stderr);
}

const char* log_last_error() { return g_last_error.c_str(); }

}  // namespace bcm3
