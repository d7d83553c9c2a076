// Device split scans of the monotone-constraint policies (see policy_scan.h). FP contraction is
// off for this translation unit: the scans must round exactly like the host oracle (g++ in ISO
// C++17 mode does not contract), so a rescan after a bound change picks the host's split.
#pragma clang fp contract(off)

#include "device/policy_scan.h"

#include <hip/hip_runtime.h>

#include "device/hip_common.h"

namespace lgap {
namespace device {

namespace {

constexpr int kPolicyThreads = 64;

// larger -= smaller, element-wise (the histogram subtraction of the host learner)
__global__ __launch_bounds__(256) void k_policy_subtract(double* __restrict__ larger, const double* __restrict__ smaller,
                                                         size_t n) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    larger[i] -= smaller[i];
  }
}

// one wave per (feature, leaf) item: the feature's group bins -> its full histogram in LDS (the
// most frequent bin filled from the leaf sums in bin order, Dataset::FeatureHistogram), then lane 0
// runs the host scan (split_math.h) against the item's bounds
__global__ __launch_bounds__(kPolicyThreads) void k_policy_scan(PolicyScanArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  double* H = reinterpret_cast<double*>(smem);            // [2 max_bin]
  int* order = reinterpret_cast<int*>(H + 2 * a.max_bin);  // [max_bin]
  const int f = blockIdx.x, r = blockIdx.y, lane = threadIdx.x;
  const size_t item = static_cast<size_t>(r) * a.F + f;
  if (!a.enable[item]) {
    if (lane == 0) {
      SplitInfo s;
      s.Reset();
      a.out[item] = s;
      a.splittable[item] = 0;
    }
    return;
  }
  const PolicyFeat fi = a.feat[f];
  const PolicyReq q = a.req[r];
  const double* gh = a.slots + static_cast<size_t>(q.slot) * a.slot_stride;
  for (int b = lane; b < fi.num_bin; b += kPolicyThreads) {
    if (b == fi.mfb) continue;
    const int k = b < fi.mfb ? b : b - 1;
    H[2 * b] = gh[2 * (fi.hist_offset + k)];
    H[2 * b + 1] = gh[2 * (fi.hist_offset + k) + 1];
  }
  __syncthreads();
  if (lane != 0) return;
  double sg = 0.0, sh = 0.0;
  for (int b = 0; b < fi.num_bin; ++b) {
    if (b == fi.mfb) continue;
    sg += H[2 * b];
    sh += H[2 * b + 1];
  }
  H[2 * fi.mfb] = q.sum_g - sg;
  H[2 * fi.mfb + 1] = q.sum_h - sh;
  FeatureScanMeta m;
  m.num_bin = fi.num_bin;
  m.default_bin = static_cast<uint32_t>(fi.default_bin);
  m.missing_type = fi.missing;
  m.bin_type = fi.bin_type;
  m.monotone = fi.monotone;
  m.penalty = fi.penalty;
  const PolicyBound pb = a.bnd[item];
  LeafBounds lb;
  lb.min = pb.min;
  lb.max = pb.max;
  SplitInfo out;
  out.Reset();
  bool sp;
  if (fi.bin_type == static_cast<int8_t>(BinType::Numerical)) {
    ThresholdBounds tb;
    const ThresholdBounds* tbp = nullptr;
    if (pb.tb_off >= 0) {
      const double* base = a.tb + pb.tb_off;
      tb.lmin = base;
      tb.lmax = base + fi.num_bin;
      tb.rmin = base + 2 * fi.num_bin;
      tb.rmax = base + 3 * fi.num_bin;
      tbp = &tb;
    }
    sp = FindBestNumerical(H, m, a.p, q.sum_g, q.sum_h, q.count, q.parent_output, lb, &out, tbp);
  } else {
    sp = FindBestCategorical(H, m, a.p, q.sum_g, q.sum_h, q.count, q.parent_output, lb, order, &out);
  }
  out.feature = sp ? f : -1;
  if (!sp) out.gain = kMinScore;
  a.out[item] = out;
  a.splittable[item] = sp ? 1 : 0;
}

}  // namespace

void LaunchPolicySubtract(double* larger, const double* smaller, size_t n, void* stream) {
  if (n == 0) return;
  const int grid = static_cast<int>(std::min<size_t>((n + 255) / 256, 2048));
  hipLaunchKernelGGL(k_policy_subtract, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), larger, smaller, n);
  HIP_CHECK(hipGetLastError());
}

void LaunchPolicyScan(const PolicyScanArgs& a, void* stream) {
  if (a.F <= 0 || a.R <= 0) return;
  const size_t lds = static_cast<size_t>(a.max_bin) * (2 * sizeof(double) + sizeof(int));
  hipLaunchKernelGGL(k_policy_scan, dim3(a.F, a.R), dim3(kPolicyThreads), lds, static_cast<hipStream_t>(stream), a);
  HIP_CHECK(hipGetLastError());
}

}  // namespace device
}  // namespace lgap
