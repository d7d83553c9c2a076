// HIP helpers for the gfx950 (CDNA4) kernels: error checks, wave64 reductions
// and scans, device buffers.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "lgap/log.h"

#define HIP_CHECK(expr)                                                                                  \
  do {                                                                                                   \
    hipError_t _e = (expr);                                                                              \
    if (_e != hipSuccess) {                                                                              \
      ::lgap::Log::Fatal("HIP error %s at %s:%d: %s", hipGetErrorName(_e), __FILE__, __LINE__, #expr); \
    }                                                                                                    \
  } while (0)

namespace lgap {
namespace device {

constexpr int kWave = 64;

// ---- wave64 primitives
__device__ __forceinline__ double WaveSum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float WaveSum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ int WaveSum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
// inclusive prefix sum across the 64 lanes
template <typename T>
__device__ __forceinline__ T WaveInclusiveScan(T v) {
  const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    T u = __shfl_up(v, o, kWave);
    if (lane >= o) v += u;
  }
  return v;
}

// ---- owning device buffer
template <typename T>
class DevBuf {
 public:
  DevBuf() = default;
  explicit DevBuf(size_t n) { Resize(n); }
  ~DevBuf() { Free(); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  void Resize(size_t n) {
    if (n == n_ && ptr_ != nullptr) return;
    if (!owns_ && ptr_ != nullptr && n <= n_) {  // views never grow in place
      n_ = n;
      return;
    }
    Free();
    n_ = n;
    if (n > 0) HIP_CHECK(hipMalloc(&ptr_, n * sizeof(T)));
  }
  void Free() {
    if (ptr_ != nullptr && owns_) (void)hipFree(ptr_);
    ptr_ = nullptr;
    n_ = 0;
    owns_ = true;
  }
  // Non-owning view into memory carved from a larger allocation (arena).
  void Attach(T* p, size_t n) {
    Free();
    ptr_ = p;
    n_ = n;
    owns_ = false;
  }
  T* get() const { return ptr_; }
  size_t size() const { return n_; }
  void Upload(const T* host, size_t n, hipStream_t s = 0) {
    if (n > n_) Resize(n);
    if (n) HIP_CHECK(hipMemcpyAsync(ptr_, host, n * sizeof(T), hipMemcpyHostToDevice, s));
  }
  void Upload(const std::vector<T>& v, hipStream_t s = 0) { Upload(v.data(), v.size(), s); }
  void Download(T* host, size_t n, hipStream_t s = 0) const {
    if (n) HIP_CHECK(hipMemcpyAsync(host, ptr_, n * sizeof(T), hipMemcpyDeviceToHost, s));
  }
  void Zero(hipStream_t s = 0) {
    if (n_) HIP_CHECK(hipMemsetAsync(ptr_, 0, n_ * sizeof(T), s));
  }

 private:
  T* ptr_ = nullptr;
  size_t n_ = 0;
  bool owns_ = true;
};

// Bump allocator laying out many small device buffers inside ONE allocation
// (one TLB reach for all per-tree state instead of a page per buffer).
class ArenaLayout {
 public:
  template <typename T>
  size_t Add(size_t count) {
    off_ = (off_ + 255) & ~static_cast<size_t>(255);
    const size_t o = off_;
    off_ += std::max<size_t>(count, 1) * sizeof(T);
    return o;
  }
  size_t bytes() const { return (off_ + 255) & ~static_cast<size_t>(255); }

 private:
  size_t off_ = 0;
};

inline int DivUp(long long a, long long b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace device
}  // namespace lgap
