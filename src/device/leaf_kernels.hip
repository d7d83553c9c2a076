// Once-per-tree leaf kernels: L1 / quantile / MAPE leaf renewal and refit leaf
// statistics (see leaf_kernels.h for the reference semantics).
#include "device/leaf_kernels.h"

#include <hip/hip_runtime.h>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include <algorithm>

#include "device/hip_common.h"
#include "lgap/log.h"

namespace lgap {
namespace device {

namespace {

constexpr int kPickThreads = 1024;

// residual of every in-bag row, leaf-major (leaf l occupies [seg_off[l], seg_off[l + 1]))
__global__ __launch_bounds__(256) void k_renew_gather(RenewArgs a, double* __restrict__ keys, float* __restrict__ vals) {
  const int leaf = blockIdx.y;
  const LeafSeg sg = a.segs[leaf];
  const int* idx = sg.buf >= 0 && sg.buf < kLeafIdxBufs ? a.idx[sg.buf] : nullptr;
  const int base = a.seg_off[leaf];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < sg.count; i += gridDim.x * blockDim.x) {
    const int row = idx ? idx[sg.start + i] : sg.start + i;
    keys[base + i] = static_cast<double>(a.label[row]) - a.score[row];
    vals[base + i] = a.weight ? a.weight[row] : 0.f;
  }
}

__device__ double BlockSumD(double v, double* sh) {
  v = WaveSum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < static_cast<int>(blockDim.x >> 6); ++i) s += sh[i];
  return s;
}

// One workgroup per leaf over its ascending-sorted residuals `v` (weights `w`): the host
// Percentile / WeightedPercentile (objectives.cpp) on the device.
__global__ __launch_bounds__(kPickThreads) void k_renew_pick(RenewArgs a, const double* __restrict__ keys,
                                                             const float* __restrict__ vals,
                                                             double* __restrict__ out, int* __restrict__ nonempty) {
  __shared__ double sh[kPickThreads / 64];
  __shared__ double s_chunk[kPickThreads];
  __shared__ int s_pos;
  __shared__ double s_cdf[2];
  const int leaf = blockIdx.x, t = threadIdx.x;
  const int n = a.segs[leaf].count;
  const double* v = keys + a.seg_off[leaf];
  const float* w = vals + a.seg_off[leaf];
  if (t == 0) nonempty[leaf] = n > 0 ? 1 : 0;
  if (n <= 1) {
    if (t == 0) out[leaf] = n == 1 ? v[0] : 0.0;
    return;
  }
  if (a.weight == nullptr) {
    if (t == 0) {
      const double fpos = static_cast<double>(n - 1) * (1.0 - a.alpha);
      const int pos = static_cast<int>(fpos) + 1;
      double r;
      if (pos < 1) {
        r = v[n - 1];  // max
      } else if (pos >= n) {
        r = v[0];      // min
      } else {
        const double bias = fpos - (pos - 1);
        const double v1 = v[n - pos], v2 = v[n - 1 - pos];  // descending positions pos - 1, pos
        r = v1 - (v1 - v2) * bias;
      }
      out[leaf] = r;
    }
    return;
  }
  // weighted: cdf over the sorted order, each thread a contiguous chunk
  const int per = (n + kPickThreads - 1) / kPickThreads;
  const int b = t * per, e = min(n, b + per);
  double cs = 0.0;
  for (int i = b; i < e; ++i) cs += static_cast<double>(w[i]);
  s_chunk[t] = cs;
  if (t == 0) s_pos = n;  // upper_bound result (n: none above thr)
  const double total = BlockSumD(cs, sh);
  const double thr = total * a.alpha;
  double base = 0.0;
  for (int i = 0; i < t; ++i) base += s_chunk[i];
  double c = base;
  for (int i = b; i < e; ++i) {
    c += static_cast<double>(w[i]);
    if (c > thr) {
      atomicMin(&s_pos, i);
      break;
    }
  }
  __syncthreads();
  const int pos = min(s_pos, n - 1);
  // cdf at pos and pos + 1 from their owners
  c = base;
  for (int i = b; i < e; ++i) {
    c += static_cast<double>(w[i]);
    if (i == pos) s_cdf[0] = c;
    if (i == pos + 1) s_cdf[1] = c;
  }
  __syncthreads();
  if (t == 0) {
    double r;
    if (pos == 0 || pos == n - 1) {
      r = v[pos];
    } else {
      const double v1 = v[pos - 1], v2 = v[pos];
      const double c0 = s_cdf[0], c1 = s_cdf[1];
      r = (c1 - c0 >= 1.0f) ? (thr - c0) / (c1 - c0) * (v2 - v1) + v1 : v2;
    }
    out[leaf] = r;
  }
}

constexpr int kRefitThreads = 256;
constexpr int kRefitLdsLeaves = 2048;

__global__ __launch_bounds__(kRefitThreads) void k_refit_partial(const float2* __restrict__ gh,
                                                                 const int* __restrict__ leaf_pred, int n, int L,
                                                                 double* __restrict__ partial) {
  __shared__ double s[3 * kRefitLdsLeaves];
  const bool lds = L <= kRefitLdsLeaves;
  double* acc = lds ? s : partial + static_cast<size_t>(blockIdx.x) * 3 * L;
  for (int i = threadIdx.x; i < 3 * L; i += blockDim.x) acc[i] = 0.0;
  __syncthreads();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int l = leaf_pred[i];
    if (l < 0 || l >= L) continue;
    const float2 v = gh[i];
    atomicAdd(&acc[3 * l], static_cast<double>(v.x));
    atomicAdd(&acc[3 * l + 1], static_cast<double>(v.y));
    atomicAdd(&acc[3 * l + 2], 1.0);
  }
  __syncthreads();
  if (lds) {
    double* dst = partial + static_cast<size_t>(blockIdx.x) * 3 * L;
    for (int i = threadIdx.x; i < 3 * L; i += blockDim.x) dst[i] = s[i];
  }
}

__global__ __launch_bounds__(256) void k_refit_fold(const double* __restrict__ partial, int nb, int L,
                                                     double* __restrict__ sums) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= 3 * L) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += partial[static_cast<size_t>(b) * 3 * L + v];
  sums[v] = s;
}

__global__ __launch_bounds__(256) void k_add_leaf_delta(double* __restrict__ score, const int* __restrict__ leaf_pred,
                                                        const double* __restrict__ delta, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) score[i] += delta[leaf_pred[i]];
}

}  // namespace

size_t RenewScratchBytes(int total, int num_leaves) {
  size_t tmp = 0;
  const int t = std::max(total, 1);
  const hipError_t e = rocprim::segmented_radix_sort_pairs(
      nullptr, tmp, static_cast<double*>(nullptr), static_cast<double*>(nullptr), static_cast<float*>(nullptr),
      static_cast<float*>(nullptr), t, std::max(num_leaves, 1), static_cast<const int*>(nullptr),
      static_cast<const int*>(nullptr), 0, 64);
  HIP_CHECK(e);
  const size_t arrays = 2 * (sizeof(double) + sizeof(float)) * static_cast<size_t>(t);
  return ((tmp + 255) & ~size_t(255)) + arrays + 1024;
}

void LaunchRenewLeaves(const RenewArgs& a, int total, void* scratch, size_t scratch_bytes, double* out, int* nonempty,
                       hipStream_t s) {
  if (a.num_leaves <= 0) return;
  const int t = std::max(total, 1);
  size_t tmp = 0;
  const hipError_t e0 = rocprim::segmented_radix_sort_pairs(
      nullptr, tmp, static_cast<double*>(nullptr), static_cast<double*>(nullptr), static_cast<float*>(nullptr),
      static_cast<float*>(nullptr), t, a.num_leaves, a.seg_off, a.seg_off + 1, 0, 64);
  HIP_CHECK(e0);
  char* p = static_cast<char*>(scratch);
  void* temp = p;
  p += (tmp + 255) & ~size_t(255);
  double* k_in = reinterpret_cast<double*>(p);
  double* k_out = k_in + t;
  float* v_in = reinterpret_cast<float*>(k_out + t);
  float* v_out = v_in + t;
  if (static_cast<size_t>(reinterpret_cast<char*>(v_out + t) - static_cast<char*>(scratch)) > scratch_bytes) {
    Log::Fatal("LaunchRenewLeaves: scratch too small");
  }
  if (total > 0) {
    const dim3 grid(std::max(1, std::min(64, DivUp(total / std::max(1, a.num_leaves), 256))), a.num_leaves);
    k_renew_gather<<<grid, 256, 0, s>>>(a, k_in, v_in);
    HIP_CHECK(hipGetLastError());
    const hipError_t e1 = rocprim::segmented_radix_sort_pairs(temp, tmp, k_in, k_out, v_in, v_out, total, a.num_leaves,
                                                              a.seg_off, a.seg_off + 1, 0, 64, s);
    HIP_CHECK(e1);
  }
  k_renew_pick<<<a.num_leaves, kPickThreads, 0, s>>>(a, k_out, v_out, out, nonempty);
  HIP_CHECK(hipGetLastError());
}

int RefitPartialBlocks(int n) { return std::max(1, std::min(512, DivUp(n, kRefitThreads * 16))); }

void LaunchRefitLeafSums(const float2* gh, const int* leaf_pred, int n, int num_leaves, double* partial, double* sums,
                         hipStream_t s) {
  const int nb = RefitPartialBlocks(n);
  k_refit_partial<<<nb, kRefitThreads, 0, s>>>(gh, leaf_pred, n, num_leaves, partial);
  HIP_CHECK(hipGetLastError());
  k_refit_fold<<<DivUp(3 * num_leaves, 256), 256, 0, s>>>(partial, nb, num_leaves, sums);
  HIP_CHECK(hipGetLastError());
}

void LaunchAddLeafDelta(double* score, const int* leaf_pred, const double* delta, int n, hipStream_t s) {
  if (n <= 0) return;
  k_add_leaf_delta<<<std::max(1, std::min(4096, DivUp(n, 256))), 256, 0, s>>>(score, leaf_pred, delta, n);
  HIP_CHECK(hipGetLastError());
}

}  // namespace device
}  // namespace lgap
