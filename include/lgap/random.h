// Bit-compatible MSVC-style LCG (reference: include/LightGBM/utils/random.h:101-111)
// so that bagging / feature-fraction / DART / EFB sampling reproduce the same
// streams for the same seeds. Usable from device code too (per-thread state).
#pragma once

#include <cmath>
#include <set>
#include <vector>

#include "lgap/meta.h"

namespace lgap {

class Random {
 public:
  LGAP_HD Random() : x_(123456789u) {}
  LGAP_HD explicit Random(int seed) : x_(static_cast<unsigned int>(seed)) {}

  LGAP_HD int NextShort(int lo, int hi) { return RandInt16() % (hi - lo) + lo; }
  LGAP_HD int NextInt(int lo, int hi) { return RandInt32() % (hi - lo) + lo; }
  LGAP_HD float NextFloat() { return static_cast<float>(RandInt16()) / 32768.0f; }

  // K sorted samples from [0, N): Bernoulli scan when dense, Floyd otherwise.
  std::vector<int> Sample(int N, int K) {
    std::vector<int> ret;
    ret.reserve(K > 0 ? K : 0);
    if (K > N || K <= 0) return ret;
    if (K == N) {
      for (int i = 0; i < N; ++i) ret.push_back(i);
      return ret;
    }
    if (K > 1 && K > (N / std::log2(K))) {
      for (int i = 0; i < N; ++i) {
        double prob = (K - static_cast<double>(ret.size())) / static_cast<double>(N - i);
        if (NextFloat() < prob) ret.push_back(i);
      }
      return ret;
    }
    std::set<int> chosen;
    for (int r = N - K; r < N; ++r) {
      int v = NextInt(0, r + 1);
      if (!chosen.insert(v).second) chosen.insert(r);
    }
    ret.assign(chosen.begin(), chosen.end());
    return ret;
  }

  LGAP_HD unsigned int state() const { return x_; }

 private:
  LGAP_HD int RandInt16() {
    x_ = 214013u * x_ + 2531011u;
    return static_cast<int>((x_ >> 16) & 0x7FFF);
  }
  LGAP_HD int RandInt32() {
    x_ = 214013u * x_ + 2531011u;
    return static_cast<int>(x_ & 0x7FFFFFFF);
  }
  unsigned int x_;
};

// Counter-based hash draw shared by the host and device GOSS samplers: the key of
// row i in iteration `iter` does not depend on thread count or visiting order.
LGAP_HD inline uint32_t Hash32(uint32_t seed, uint32_t i) {
  uint32_t x = i * 0x9E3779B1u ^ (seed * 0x85EBCA77u + 0x165667B1u);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
LGAP_HD inline uint32_t GossSeed(int bagging_seed, int iter) {
  return static_cast<uint32_t>(bagging_seed) * 0x9E3779B9u + static_cast<uint32_t>(iter) * 0x85EBCA6Bu;
}
// GOSS works on fixed row tiles (host and device alike).
constexpr int kGossTile = 4096;

}  // namespace lgap
