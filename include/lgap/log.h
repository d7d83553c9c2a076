// Leveled logging with an optional redirect callback (used by the Python
// binding's register_logger). Fatal throws std::runtime_error so the C API can
// turn it into a -1 return + LGBM_GetLastError, matching utils/log.h:40-185.
#pragma once

#include <cstdarg>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace lgap {

enum class LogLevel : int { Fatal = -1, Warning = 0, Info = 1, Debug = 2 };

class Log {
 public:
  using Callback = void (*)(const char*);
  static void ResetLevel(LogLevel level) { level_() = level; }
  static LogLevel Level() { return level_(); }
  static void ResetCallback(Callback cb) { callback_() = cb; }

  static void Debug(const char* fmt, ...) {
    va_list a; va_start(a, fmt); Write(LogLevel::Debug, "Debug", fmt, a); va_end(a);
  }
  static void Info(const char* fmt, ...) {
    va_list a; va_start(a, fmt); Write(LogLevel::Info, "Info", fmt, a); va_end(a);
  }
  static void Warning(const char* fmt, ...) {
    va_list a; va_start(a, fmt); Write(LogLevel::Warning, "Warning", fmt, a); va_end(a);
  }
  [[noreturn]] static void Fatal(const char* fmt, ...) {
    char buf[2048];
    va_list a; va_start(a, fmt); vsnprintf(buf, sizeof(buf), fmt, a); va_end(a);
    if (level_() >= LogLevel::Fatal) {
      std::string line = std::string("[LambdaGap] [Fatal] ") + buf + "\n";
      Emit(line.c_str());
    }
    throw std::runtime_error(std::string(buf));
  }

 private:
  static void Emit(const char* s) {
    if (callback_() != nullptr) {
      callback_()(s);
    } else {
      fputs(s, stdout);
      fflush(stdout);
    }
  }
  static void Write(LogLevel lv, const char* tag, const char* fmt, va_list a) {
    if (static_cast<int>(lv) > static_cast<int>(level_())) return;
    char buf[4096];
    vsnprintf(buf, sizeof(buf), fmt, a);
    std::string line = std::string("[LambdaGap] [") + tag + "] " + buf + "\n";
    Emit(line.c_str());
  }
  static LogLevel& level_() { static LogLevel l = LogLevel::Info; return l; }
  static Callback& callback_() { static Callback c = nullptr; return c; }
};

#define LGAP_CHECK(cond) \
  if (!(cond)) ::lgap::Log::Fatal("Check failed: " #cond " at %s, line %d", __FILE__, __LINE__)
#define LGAP_CHECK_EQ(a, b) LGAP_CHECK((a) == (b))
#define LGAP_CHECK_NE(a, b) LGAP_CHECK((a) != (b))
#define LGAP_CHECK_GE(a, b) LGAP_CHECK((a) >= (b))
#define LGAP_CHECK_LE(a, b) LGAP_CHECK((a) <= (b))
#define LGAP_CHECK_GT(a, b) LGAP_CHECK((a) > (b))
#define LGAP_CHECK_LT(a, b) LGAP_CHECK((a) < (b))

}  // namespace lgap
