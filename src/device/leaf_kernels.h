// Per-leaf device kernels that run once per tree (not per split):
//  * L1 / quantile / MAPE leaf renewal: each leaf's output becomes a (weighted)
//    percentile of its in-bag residuals label - score (reference
//    serial_tree_learner.cpp:924-962 RenewTreeOutput, CUDA twin
//    cuda_regression_objective.cu:151,370): residuals gathered leaf-major,
//    segment-sorted on the device (rocPRIM segmented radix sort, stable), one
//    workgroup per leaf picks the percentile with the host's interpolation;
//  * refit (reference serial_tree_learner.cpp:247-286 FitByExistingTree, CUDA twin
//    cuda_single_gpu_tree_learner.cu:19-78 ReduceLeafStatKernel /
//    CalcRefitLeafOutputKernel): per-leaf gradient / hessian / count sums over a
//    leaf assignment, and the score delta of the refitted outputs.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace lgap {
namespace device {

struct LeafSeg {
  int buf;    // index buffer of the leaf's rows (-1: identity rows)
  int start;  // first position in that buffer
  int count;  // rows
  int pad;
};

constexpr int kLeafIdxBufs = 8;  // >= kFrontierIdx (frontier.h)

struct RenewArgs {
  const double* score;  // class slice of the device score
  const float* label;
  const float* weight;  // per-row percentile weights (sample weights or MAPE label weights), nullptr: none
  const int* idx[kLeafIdxBufs];  // row-index buffers by id (0/1 ping-pong, 2 bag, 3+ frontier depth buffers)
  const LeafSeg* segs;  // [num_leaves]
  const int* seg_off;   // [num_leaves + 1] offsets of the leaves in the gathered arrays
  int num_leaves;
  double alpha;         // percentile (0.5: L1 / MAPE)
};

// Scratch bytes for `total` gathered residuals over `num_leaves` leaves.
size_t RenewScratchBytes(int total, int num_leaves);
// out[leaf] = renewed output; nonempty[leaf] = 1 when the leaf had rows.
void LaunchRenewLeaves(const RenewArgs& a, int total, void* scratch, size_t scratch_bytes, double* out, int* nonempty,
                       hipStream_t s);

// sums[3 * l + {0, 1}] = (sum g, sum h), cnt[l] = rows of leaf l over leaf_pred (all n rows);
// `partial` holds blocks x num_leaves x 3 doubles (see RefitPartialBlocks)
int RefitPartialBlocks(int n);
void LaunchRefitLeafSums(const float2* gh, const int* leaf_pred, int n, int num_leaves, double* partial, double* sums,
                         hipStream_t s);
// score[i] += delta[leaf_pred[i]]
void LaunchAddLeafDelta(double* score, const int* leaf_pred, const double* delta, int n, hipStream_t s);

}  // namespace device
}  // namespace lgap
