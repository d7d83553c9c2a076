// Linear-leaf trees on the device (reference linear_tree_learner.cpp:180-360 CalculateLinear):
// per leaf, the Gram system of a ridge-regularised Newton step over the numerical features on
// the leaf's branch plus a constant,
//     A = sum_i h_i x_i x_i^T,   c = sum_i g_i x_i      (x_i = [raw features of row i, 1])
// accumulated with fp64 MFMA (v_mfma_f64_16x16x4f64: four rows per instruction, the 16x16
// tiles of [A | c] in accumulator registers), rows with a NaN in any of the leaf's features
// left out. The small systems are solved on the host (Cholesky, learner/linear_solve.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device/leaf_kernels.h"

namespace lgap {
namespace device {

constexpr int kLinMaxM = 63;  // unknowns per leaf: <= 62 branch features + the constant
constexpr int kLinDim = 64;   // [A | c] in up to four 16-wide tiles per dimension (c = column m)

struct LinearGramArgs {
  const float* raw;          // [N][F] raw values of the inner features
  int F;
  const float2* gh;          // (g, h) of the tree's class
  const int* idx[kLeafIdxBufs];
  const LeafSeg* segs;       // [num_leaves] the leaf's rows
  const int* feat_off;       // [num_leaves + 1] offsets into feats
  const int* feats;          // the leaves' branch features (inner indices), sorted
  int num_leaves;
  int chunks;                // row chunks per leaf (grid.x)
};

// out[leaf][kLinDim][kLinDim]: A (m x m, both triangles) in rows / columns [0, m), c in column
// m; usable[leaf]: the reference's "enough data" count with NaNs in the dataset (non-NaN values
// read before a row's first NaN). partial: chunks x num_leaves x (kLinDim^2 + 1) doubles.
size_t LinearGramPartialDoubles(int num_leaves, int chunks);
void LaunchLinearGram(const LinearGramArgs& a, int max_m, double* partial, double* out, long long* usable,
                      hipStream_t s);

// Linear leaf values for the score update (traverse_kernels.h LaunchTraverseLinear)
struct LinearLeaves {
  const float* raw;      // [N][F] raw values (inner features)
  int F;
  const int* off;        // [num_leaves + 1] offsets into feat / coef
  const int* feat;       // inner features of each leaf's model
  const double* coef;    // their coefficients
  const double* cnst;    // [num_leaves] the models' constants
};

}  // namespace device
}  // namespace lgap
