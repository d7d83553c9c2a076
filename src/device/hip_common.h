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

// ---- DPP wave64 primitives (gfx9 data-parallel-primitive moves: row_shr:n = 0x110 + n,
// row_bcast:15 = 0x142, row_bcast:31 = 0x143). A DPP move is a VALU operand modifier:
// a few cycles per step instead of a ds_bpermute round trip through the LDS crossbar.
template <int kCtrl>
__device__ __forceinline__ int DppMove(int v) {
  return __builtin_amdgcn_update_dpp(0, v, kCtrl, 0xf, 0xf, false);
}
template <int kCtrl>
__device__ __forceinline__ float DppMove(float v) {
  return __int_as_float(DppMove<kCtrl>(__float_as_int(v)));
}
template <int kCtrl>
__device__ __forceinline__ double DppMove(double v) {
  const int lo = DppMove<kCtrl>(__double2loint(v));
  const int hi = DppMove<kCtrl>(__double2hiint(v));
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double ReadLane(double v, int lane) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), lane),
                          __builtin_amdgcn_readlane(__double2loint(v), lane));
}
__device__ __forceinline__ int ReadLane(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

// Inclusive wave scan with an associative op: Hillis-Steele inside each 16-lane row
// (row_shr 1, 2, 4, 8), then row 15 -> rows 1 and 3 (row_bcast:15) and lane 31 -> rows 2
// and 3 (row_bcast:31).
template <typename T, typename Op>
__device__ __forceinline__ T WaveScanDpp(T v, Op op) {
  const int lane = threadIdx.x & 63, rl = lane & 15;
  T t = DppMove<0x111>(v);
  if (rl >= 1) v = op(v, t);
  t = DppMove<0x112>(v);
  if (rl >= 2) v = op(v, t);
  t = DppMove<0x114>(v);
  if (rl >= 4) v = op(v, t);
  t = DppMove<0x118>(v);
  if (rl >= 8) v = op(v, t);
  t = DppMove<0x142>(v);
  if (lane & 16) v = op(v, t);
  t = DppMove<0x143>(v);
  if (lane >= 32) v = op(v, t);
  return v;
}
template <typename T>
__device__ __forceinline__ T WaveInclusiveSumDpp(T v) {
  return WaveScanDpp(v, [](T x, T y) { return x + y; });
}
// wave maximum, the same value in every lane
__device__ __forceinline__ double WaveMaxDpp(double v) {
  return ReadLane(WaveScanDpp(v, [](double x, double y) { return x > y ? x : y; }), 63);
}
__device__ __forceinline__ int WaveMaxDpp(int v) {
  return ReadLane(WaveScanDpp(v, [](int x, int y) { return x > y ? x : y; }), 63);
}
// Lane of the wave's best (g descending, then x ascending, then y ascending): one DPP
// max per key and a ballot, the winner's payload is then read with ReadLane.
__device__ __forceinline__ int WaveArgBestLane(double g, int x, int y) {
  const double mg = WaveMaxDpp(g);
  const bool t1 = g == mg;
  const int mx = -WaveMaxDpp(t1 ? -x : -0x7fffffff - 1);
  const bool t2 = t1 && x == mx;
  const int my = -WaveMaxDpp(t2 ? -y : -0x7fffffff - 1);
  const unsigned long long m = __ballot(t2 && y == my);
  return m ? __ffsll(static_cast<long long>(m)) - 1 : 0;
}

// ---- wave64 reductions / scans (on the DPP primitives above)
__device__ __forceinline__ double WaveSum(double v) { return ReadLane(WaveInclusiveSumDpp(v), 63); }
__device__ __forceinline__ float WaveSum(float v) {
  return __int_as_float(ReadLane(__float_as_int(WaveScanDpp(v, [](float x, float y) { return x + y; })), 63));
}
__device__ __forceinline__ int WaveSum(int v) { return ReadLane(WaveInclusiveSumDpp(v), 63); }
// 64-bit integer wave sum (butterfly: the total in every lane)
__device__ __forceinline__ long long WaveSumLL(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
// inclusive prefix sum across the 64 lanes
template <typename T>
__device__ __forceinline__ T WaveInclusiveScan(T v) {
  return WaveInclusiveSumDpp(v);
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
  // Take ownership of a device allocation of n elements (hipMalloc'd elsewhere).
  void Adopt(T* p, size_t n) {
    Free();
    ptr_ = p;
    n_ = n;
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
  // Copies are issued in chunks of at most kCopyChunk bytes: a single pageable copy of more
  // than 4 GiB (rowbins / colbins of a wide 10M-row dataset) arrived incomplete on MI355X.
  static constexpr size_t kCopyChunk = size_t(1) << 30;
  void Upload(const T* host, size_t n, hipStream_t s = 0) {
    if (n > n_) Resize(n);
    const char* src = reinterpret_cast<const char*>(host);
    char* dst = reinterpret_cast<char*>(ptr_);
    for (size_t off = 0, bytes = n * sizeof(T); off < bytes; off += kCopyChunk) {
      HIP_CHECK(hipMemcpyAsync(dst + off, src + off, std::min(kCopyChunk, bytes - off), hipMemcpyHostToDevice, s));
    }
  }
  void Upload(const std::vector<T>& v, hipStream_t s = 0) { Upload(v.data(), v.size(), s); }
  void Download(T* host, size_t n, hipStream_t s = 0) const {
    char* dst = reinterpret_cast<char*>(host);
    const char* src = reinterpret_cast<const char*>(ptr_);
    for (size_t off = 0, bytes = n * sizeof(T); off < bytes; off += kCopyChunk) {
      HIP_CHECK(hipMemcpyAsync(dst + off, src + off, std::min(kCopyChunk, bytes - off), hipMemcpyDeviceToHost, s));
    }
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
