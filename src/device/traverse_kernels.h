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

#include "device/leaf_kernels.h"
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

// Score update from the final leaf ranges of the frontier tree just grown (reference
// serial_tree_learner.cpp AddPredictionToScore via data_partition_, CUDA twin
// cuda_data_partition.cu AddPredictionToScoreKernel), when every row sits in exactly one
// leaf's row-index segment (no bagging). Instead of walking the tree over the packed rows:
//  LaunchLeafMap   a first pass finds where each leaf's rows (monotone along the segment: the
//                  frontier partition's left / right placement) cross every kLTRows-row tile
//                  boundary; then one block per tile gathers the tile's row -> leaf map into
//                  LDS from those runs and writes it out coalesced (uint8 <= 256 leaves, else
//                  uint16). No scattered global writes; the leaf values are copied to lv_out.
//  LaunchLeafMapAdd       score[i] += lv[map[i]] (deferred by the learner until the score is read)
//  LaunchLeafMapAddGrad   the same fused with the next iteration's pointwise gradients
constexpr int kLTShift = 12, kLTRows = 1 << kLTShift;
constexpr int kLMMaxLeaves = 1024;  // larger trees take the traversal
struct LeafMapArgs {
  const int* idx[kLeafIdxBufs];  // row-index buffers by id (LeafSeg::buf; -1: identity rows)
  const LeafSeg* segs;           // [num_leaves]; pad bit 0: the segment's rows descend
  const int* seg_off;            // [num_leaves + 1] leaf-major positions of the segments
  const double* leaf_value;      // [num_leaves]
  int num_leaves;
  int n;                         // rows == seg_off[num_leaves]
};
// ints of the tile-bounds scratch for n rows and num_leaves leaves
size_t LeafTileBoundsInts(int n, int num_leaves);
// Bagged / GOSS trees (reference gbdt.cpp:495-516 UpdateScore: the in-bag rows take their leaf
// from the learner's partition, only the out-of-bag rows walk the tree): LaunchLeafMap runs over
// the leaves' segments plus one more, the ascending out-of-bag list (LeafMapArgs::idx
// [kLeafOobBuf]) as a placeholder leaf num_leaves - 1 of value 0; LaunchLeafMapList then walks
// the listed rows through the compact tree and overwrites their map entries with their leaves.
// colbins != nullptr: the group-major copy colbins[g * n + row], else the packed rows.
// map_leaves: the leaf count the map was built for (uint8 entries up to 256, else uint16).
// rows_per_thread (2 / 4 / 8): independent walks per lane (the gathers of a deep level are
// latency-bound: more walks in flight).
constexpr int kLeafOobBuf = kLeafIdxBufs - 1;
void LaunchLeafMapList(const uint8_t* colbins, const uint32_t* rowbins, int stride_dw, int width, int n,
                       const int* list, int count, const TNode* nodes, int num_nodes, const TCat* cats,
                       const uint32_t* cat_bits, int map_leaves, void* map, int rows_per_thread, int num_cu,
                       hipStream_t s);
void LaunchLeafMap(const LeafMapArgs& a, int* bounds, void* map, double* lv_out, hipStream_t s);
void LaunchLeafMapAdd(const void* map, const double* lv, int num_leaves, int n, double* score, int num_cu,
                      hipStream_t s);
void LaunchLeafMapAddGrad(const void* map, const double* lv, int num_leaves, int n, double* score,
                          const PointwiseParams& p, const float* label, const float* weight, const float* aux, float2* gh,
                          int num_cu, hipStream_t s);

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
