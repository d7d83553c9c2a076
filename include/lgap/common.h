// String / numeric / bitset helpers and the phase timer (reference analogue:
// include/LightGBM/utils/common.h, Timer at :984-1068). Locale independent
// number formatting is done with snprintf("%g"/"%.17g") which matches the
// reference's fmt "{:g}"/"{:.17g}" output for the model text format.
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "lgap/log.h"
#include "lgap/meta.h"

namespace lgap {
namespace common {

inline std::string Trim(std::string s) {
  const char* ws = " \t\n\r\f\v";
  size_t b = s.find_first_not_of(ws);
  if (b == std::string::npos) return "";
  size_t e = s.find_last_not_of(ws);
  return s.substr(b, e - b + 1);
}

inline std::string RemoveQuotes(std::string s) {
  s = Trim(s);
  if (s.size() >= 2 && ((s.front() == '"' && s.back() == '"') || (s.front() == '\'' && s.back() == '\''))) {
    return s.substr(1, s.size() - 2);
  }
  return s;
}

inline std::vector<std::string> Split(const std::string& s, char delim) {
  std::vector<std::string> out;
  size_t start = 0;
  for (size_t i = 0; i <= s.size(); ++i) {
    if (i == s.size() || s[i] == delim) {
      if (i > start) out.emplace_back(s.substr(start, i - start));
      start = i + 1;
    }
  }
  return out;
}

inline std::vector<std::string> SplitAny(const std::string& s, const char* delims) {
  std::vector<std::string> out;
  size_t start = 0;
  for (size_t i = 0; i <= s.size(); ++i) {
    if (i == s.size() || std::strchr(delims, s[i]) != nullptr) {
      if (i > start) out.emplace_back(s.substr(start, i - start));
      start = i + 1;
    }
  }
  return out;
}

inline std::vector<std::string> SplitLines(const char* s) {
  std::vector<std::string> out;
  const char* p = s;
  while (*p) {
    const char* q = p;
    while (*q && *q != '\n' && *q != '\r') ++q;
    out.emplace_back(p, q - p);
    while (*q == '\n' || *q == '\r') ++q;
    p = q;
  }
  return out;
}

inline bool StartsWith(const std::string& s, const std::string& p) {
  return s.size() >= p.size() && s.compare(0, p.size(), p) == 0;
}

inline std::string ToLower(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

// Fast, locale-free double parser; accepts nan/inf/na/null tokens.
inline const char* Atof(const char* p, double* out) {
  while (*p == ' ' || *p == '\t') ++p;
  const char* start = p;
  char* end = nullptr;
  double v = std::strtod(p, &end);
  if (end == p) {
    // textual tokens
    std::string tok;
    while (*p && *p != ',' && *p != '\t' && *p != ' ' && *p != '\n' && *p != '\r' && *p != ':') tok.push_back(*p++);
    std::string l = ToLower(tok);
    if (l == "na" || l == "nan" || l == "null" || l.empty() || l == "none") {
      *out = NAN;
    } else if (l == "inf" || l == "infinity" || l == "+inf") {
      *out = 1e300;
    } else if (l == "-inf" || l == "-infinity") {
      *out = -1e300;
    } else {
      Log::Fatal("Unknown token %s in data file", tok.c_str());
    }
    (void)start;
    return p;
  }
  *out = v;
  return end;
}

inline double AtofOrDie(const std::string& s) {
  double v;
  const char* e = Atof(s.c_str(), &v);
  while (*e == ' ') ++e;
  if (*e != '\0') Log::Fatal("Cannot parse '%s' as a number", s.c_str());
  return v;
}

inline int AtoiOrDie(const std::string& s) {
  char* end = nullptr;
  long v = std::strtol(s.c_str(), &end, 10);
  if (end == s.c_str()) Log::Fatal("Cannot parse '%s' as an integer", s.c_str());
  return static_cast<int>(v);
}

template <typename T>
inline std::string Join(const std::vector<T>& v, const char* sep) {
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) ss << sep;
    ss << v[i];
  }
  return ss.str();
}

inline std::string FormatG(double v) {
  char buf[48];
  snprintf(buf, sizeof(buf), "%g", v);
  return buf;
}
inline std::string Format17(double v) {
  char buf[48];
  snprintf(buf, sizeof(buf), "%.17g", v);
  return buf;
}

// Array -> space separated string, identical to the reference model format.
template <bool HighPrecision = false, typename T>
inline std::string ArrayToString(const std::vector<T>& arr, size_t n) {
  std::string out;
  n = std::min(n, arr.size());
  out.reserve(n * 8);
  for (size_t i = 0; i < n; ++i) {
    if (i) out.push_back(' ');
    if constexpr (std::is_floating_point<T>::value) {
      out += HighPrecision ? Format17(static_cast<double>(arr[i])) : FormatG(static_cast<double>(arr[i]));
    } else {
      out += std::to_string(static_cast<long long>(arr[i]));
    }
  }
  return out;
}

template <typename T>
inline std::vector<T> StringToArray(const std::string& s, size_t n_expected = 0) {
  std::vector<T> out;
  if (n_expected) out.reserve(n_expected);
  const char* p = s.c_str();
  while (*p) {
    while (*p == ' ') ++p;
    if (!*p) break;
    double v;
    p = Atof(p, &v);
    out.push_back(static_cast<T>(v));
  }
  return out;
}

inline int RoundInt(double x) { return static_cast<int>(x + 0.5f); }

template <typename T>
inline int Sign(T x) { return (x > T(0)) - (x < T(0)); }

inline double AvoidInf(double x) {
  if (std::isnan(x)) return 0.0;
  if (x >= 1e300) return 1e300;
  if (x <= -1e300) return -1e300;
  return x;
}

inline float AvoidInf(float x) {
  if (std::isnan(x)) return 0.0f;
  if (x >= 1e38f) return 1e38f;
  if (x <= -1e38f) return -1e38f;
  return x;
}

inline void Softmax(std::vector<double>* p) {
  double wmax = (*p)[0];
  for (size_t i = 1; i < p->size(); ++i) wmax = std::max(wmax, (*p)[i]);
  double s = 0.0;
  for (auto& v : *p) { v = std::exp(v - wmax); s += v; }
  for (auto& v : *p) v /= s;
}

inline void Softmax(const double* in, double* out, int n) {
  double wmax = in[0];
  for (int i = 1; i < n; ++i) wmax = std::max(wmax, in[i]);
  double s = 0.0;
  for (int i = 0; i < n; ++i) { out[i] = std::exp(in[i] - wmax); s += out[i]; }
  for (int i = 0; i < n; ++i) out[i] /= s;
}

// Bitset helpers for categorical thresholds (uint32 words).
inline std::vector<uint32_t> ConstructBitset(const int* vals, int n) {
  std::vector<uint32_t> ret;
  for (int i = 0; i < n; ++i) {
    int i1 = vals[i] / 32, i2 = vals[i] % 32;
    if (static_cast<int>(ret.size()) < i1 + 1) ret.resize(i1 + 1, 0);
    ret[i1] |= (1u << i2);
  }
  return ret;
}

LGAP_HD inline bool FindInBitset(const uint32_t* bits, int n, int pos) {
  int i1 = pos / 32;
  if (i1 >= n) return false;
  int i2 = pos % 32;
  return (bits[i1] >> i2) & 1;
}

inline double GetDoubleUpperBound(double a) { return std::nextafter(a, INFINITY); }
inline bool CheckDoubleEqualOrdered(double a, double b) { return b <= std::nextafter(a, INFINITY); }

// Returns the arg max; ties resolve to the lowest index (array_args.h semantics).
template <typename T>
inline size_t ArgMax(const std::vector<T>& v) {
  if (v.empty()) return 0;
  size_t best = 0;
  for (size_t i = 1; i < v.size(); ++i) if (v[i] > v[best]) best = i;
  return best;
}

inline int NumThreads();

}  // namespace common

// ---------------------------------------------------------------------------
// Phase timer: always compiled (cheap atomic adds); printed when
// LGAP_TIMETAG=1 is in the environment (reference: USE_TIMETAG/global_timer).
class PhaseTimer {
 public:
  static PhaseTimer& Global() { static PhaseTimer t; return t; }
  bool enabled() const { return enabled_; }
  void Add(const char* name, double seconds) {
    std::lock_guard<std::mutex> lk(mu_);
    auto& e = stats_[name];
    e.first += seconds;
    e.second += 1;
  }
  std::string Report() const {
    std::lock_guard<std::mutex> lk(mu_);
    std::stringstream ss;
    for (auto& kv : stats_) {
      char buf[256];
      snprintf(buf, sizeof(buf), "%-40s %10.4f s  %8lld calls\n", kv.first.c_str(), kv.second.first,
               static_cast<long long>(kv.second.second));
      ss << buf;
    }
    return ss.str();
  }
  void Reset() { std::lock_guard<std::mutex> lk(mu_); stats_.clear(); }
  ~PhaseTimer() {
    if (enabled_ && !stats_.empty()) fprintf(stderr, "[LambdaGap] phase timings:\n%s", Report().c_str());
  }

 private:
  PhaseTimer() {
    const char* e = getenv("LGAP_TIMETAG");
    enabled_ = e != nullptr && e[0] == '1';
  }
  bool enabled_ = false;
  mutable std::mutex mu_;
  std::map<std::string, std::pair<double, long long>> stats_;
};

// Every ScopedTimer phase is also a roctx range ("lgap:<phase>"), so
// `rocprofv3 --marker-trace` lines the phases up with the kernel trace
// (SURVEY.md 5.1). roctx calls are no-ops unless a profiler is attached.
class ScopedTimer {
 public:
  explicit ScopedTimer(const char* name) : name_(name) {
    roctxRangePushA(name);
    if (PhaseTimer::Global().enabled()) start_ = std::chrono::steady_clock::now();
  }
  ~ScopedTimer() {
    roctxRangePop();
    if (PhaseTimer::Global().enabled()) {
      auto d = std::chrono::duration<double>(std::chrono::steady_clock::now() - start_).count();
      PhaseTimer::Global().Add(name_, d);
    }
  }

 private:
  const char* name_;
  std::chrono::steady_clock::time_point start_;
};

}  // namespace lgap
