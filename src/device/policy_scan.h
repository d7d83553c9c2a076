// Device split scans for the tree-growth policies whose bookkeeping is sequential and tiny but
// whose scans are not: intermediate / advanced monotone constraints (reference
// monotone_constraints.hpp:516-857 IntermediateLeafConstraints, :858-1186
// AdvancedLeafConstraints; serial_tree_learner.cpp:1010-1060 RecomputeBestSplitForLeaf).
//
// The leaves' histograms stay resident on the device (one fp64 slot of 2 x num_total_bin per
// leaf, built by the HIP histogram kernels, larger child = parent - smaller in place); after
// every split the host walks the tree (a few dozen nodes), tightens the affected leaves' output
// bounds and asks for a rescan of exactly those leaves. One launch scans every (leaf, feature)
// of the batch against its bounds -- flat [min, max] per leaf (intermediate) or per-threshold
// child bounds (advanced, ThresholdBounds arrays) -- and only the SplitInfo records come back
// (F x ~100 bytes per leaf instead of the 2 x TB doubles of a histogram download).
//
// Numerics: each (leaf, feature) item runs the host oracle of split_math.h
// (FindBestNumerical / FindBestCategorical) over the feature's full histogram in LDS, with FP
// contraction off, so a device scan returns bit for bit what the host learner's scan of the same
// histogram returns.
#pragma once

#include <cstdint>

#include "lgap/split_math.h"

namespace lgap {
namespace device {

struct PolicyFeat {
  int hist_offset, num_bin, mfb, default_bin;
  int8_t missing, bin_type, monotone, pad;
  double penalty;
};

// one leaf of a scan batch: its histogram slot and statistics
struct PolicyReq {
  int slot, count;
  double sum_g, sum_h, parent_output;
};

// bounds of one (leaf, feature) item: flat [min, max], or (tb_off >= 0) the ThresholdBounds
// arrays lmin, lmax, rmin, rmax (num_bin doubles each) at tb[tb_off]
struct PolicyBound {
  double min, max;
  long long tb_off;
};

struct PolicyScanArgs {
  const double* slots;
  size_t slot_stride;     // doubles per slot (2 x num_total_bin)
  const PolicyFeat* feat;
  int F, R, max_bin;
  const PolicyReq* req;   // [R]
  const PolicyBound* bnd; // [R][F]
  const uint8_t* enable;  // [R][F] 0: the feature is not scanned for this leaf
  const double* tb;
  SplitParams p;
  SplitInfo* out;         // [R][F]
  uint8_t* splittable;    // [R][F]
};

// larger slot -= smaller slot (2 x TB doubles), then the scans of the batch
void LaunchPolicySubtract(double* larger, const double* smaller, size_t n, void* stream);
void LaunchPolicyScan(const PolicyScanArgs& a, void* stream);

}  // namespace device
}  // namespace lgap
