// Score update by tree traversal over packed rows (reference tree.cpp:153-318
// AddPredictionToScore over binned data; cuda_tree.cu:317 AddPredictionToScoreKernel).
//
// Each numerical node's predicate is precomputed in GROUP-bin space, so a level is one
// 16-byte LDS node read, one byte of the staged row and three integer compares (no per-row
// decode of the feature bin): with lo/hi the group bins of the feature's stored bins,
//   gb outside [lo, hi]  -> the most frequent bin: `out_left`
//   gb == gmiss          -> the missing bin (zero / NaN): `default_left`
//   otherwise            -> gb <= tg  (tg: the last group bin whose feature bin <= threshold)
// exactly the decision of GoLeft (split_scan.h) on the decoded bin. Categorical nodes keep
// the decode + bitset path.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "lgap/pointwise.h"

namespace lgap {
namespace device {

struct TNode {
  uint16_t group, lo, hi, tg;
  int16_t gmiss;   // -1: no separate missing bin in range
  uint8_t flags;   // bit0 out_left, bit1 default_left, bit2 categorical
  uint8_t pad;
  int16_t left, right;  // >= 0: node, < 0: ~leaf
};
static_assert(sizeof(TNode) == 16, "TNode layout");

// categorical node data, indexed by node (meaningful for categorical nodes only)
struct TCat {
  int offset, num_bin, mfb, begin, nwords, pad;
};

constexpr uint8_t kTOutLeft = 1, kTDefaultLeft = 2, kTCat = 4;

// score[i] += value of row i's leaf, rows [0, n) of the packed matrix (stride_dw dwords/row)
// 4-bit copy of 8-bit packed rows whose every group has <= 16 bins (max_bin <= 15 data):
// out[row * stride4 + d] holds groups 8d..8d+7 as nibbles (reference dense_bin.hpp:18-97
// IS_4BIT). Read by the frontier histograms (hist_nib) and the training score update (width 0).
void LaunchPackNibbles(const uint32_t* rowbins, int stride_dw, int n, int groups, uint32_t* out, int stride4,
                       hipStream_t s);

// width: 0 = 4-bit rows, 1 = 8-bit, 2 = 16-bit group bins
void LaunchTraverse(const uint32_t* rowbins, int stride_dw, int width, int n, const TNode* nodes, int num_nodes,
                    const TCat* cats, const uint32_t* cat_bits, const double* leaf_value, int num_leaves, double* score,
                    int num_cu, hipStream_t s);

// the traversal fused with the next iteration's pointwise gradients (lgap/pointwise.h): score[i]
// += leaf value, then gh[i] = gradient / hessian at the new score (one pass over the rows instead
// of a traversal and a gradient kernel)
void LaunchTraverseGrad(const uint32_t* rowbins, int stride_dw, int width, int n, const TNode* nodes, int num_nodes,
                        const TCat* cats, const uint32_t* cat_bits, const double* leaf_value, int num_leaves,
                        double* score, const PointwiseParams& p, const float* label, const float* weight,
                        const float* aux, float2* gh, int num_cu, hipStream_t s);

// linear-leaf trees (linear_kernels.h LinearLeaves): score[i] += the leaf's linear model at
// row i's raw values (its constant output when one of them is NaN); 8- / 16-bit rows
struct LinearLeaves;
void LaunchTraverseLinear(const uint32_t* rowbins, int stride_dw, int width, int n, const TNode* nodes, int num_nodes,
                          const TCat* cats, const uint32_t* cat_bits, const double* leaf_value, int num_leaves,
                          const LinearLeaves& lin, double* score, int num_cu, hipStream_t s);

// the same over the group-major copy colbins[g * n + row] (wide training rows)
void LaunchTraverseCols(const uint8_t* colbins, int width, int n, const TNode* nodes, int num_nodes, const TCat* cats,
                        const uint32_t* cat_bits, const double* leaf_value, int num_leaves, double* score, int num_cu,
                        hipStream_t s);

}  // namespace device
}  // namespace lgap
