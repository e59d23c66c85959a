// log.h -- printf-style logging in the spirit of bcm3::Logger (src/utils/Logger.h:5-50).
#pragma once
#include <cstdarg>
#include <string>

namespace bcm3 {

enum class LogLevel { Info = 0, Warning = 1, Error = 2, Silent = 3 };

void log_set_level(LogLevel console_level);
void log_message(LogLevel level, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
// last error message (exposed through the C API's bcm3_last_error)
const char* log_last_error();

}  // namespace bcm3

#define LOG(...) ::bcm3::log_message(::bcm3::LogLevel::Info, __VA_ARGS__)
#define LOGWARNING(...) ::bcm3::log_message(::bcm3::LogLevel::Warning, __VA_ARGS__)
#define LOGERROR(...) ::bcm3::log_message(::bcm3::LogLevel::Error, __VA_ARGS__)
