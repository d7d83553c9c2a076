// Device-resident row sampling for the HIP learner: bagging (uniform and
// balanced pos/neg) and GOSS, written straight into the learner's bag index
// list so the gradients never leave HBM.
//
//  * bagging draws the SAME bag as the host SampleStrategy (and the reference,
//    bagging.hpp:230-270): row i uses the (i % 1024 + 1)-th draw of the LCG
//    Random(bagging_seed + i / 1024), continued across re-bags. Each thread jumps
//    its block's stream ahead with a precomputed (a^j, c_j) table instead of
//    stepping sequentially, and every re-bag advances the per-block states.
//  * GOSS (goss.hpp:118-167) works per 4096-row tile: the top `top_rate` rows by
//    sum_k |g_k * h_k| are kept (threshold = exact k-th largest, radix-selected
//    in LDS), an exact-size uniform sample of `other_rate` rows is drawn from the
//    rest (the `other_k` smallest hash keys, again radix-selected) and their
//    (g, h) are scaled by (cnt - top_k) / other_k in place.
// Both end in one stable compaction (ascending row order) into `out`.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace lgap {
namespace device {

constexpr int kSampleTile = 4096;       // rows per workgroup (256 threads x 16 rows) == lgap::kGossTile
constexpr int kSampleRandBlock = 1024;  // rows per bagging Random stream (SampleStrategy kRandBlock)

struct SampleArgs {
  int mode = 0;  // 1 bagging, 2 balanced bagging, 3 GOSS, 4 bagging by query
  int N = 0;
  int K = 1;  // classes (GOSS sums |g*h| over them and scales all of them)
  double fraction = 1.0, pos_fraction = 1.0, neg_fraction = 1.0;
  double top_rate = 0.2, other_rate = 0.1;
  uint32_t seed = 0;             // GOSS hash seed (changes every iteration)
  const float* label = nullptr;  // balanced bagging
  float2* gh = nullptr;          // GOSS: class-major (g, h), scaled in place
  unsigned* rng = nullptr;       // bagging: one LCG state per 1024-row block (advanced by the scatter)
                                 // (by query: per 1024-query block, advanced by LaunchSampleAdvanceUnits)
  const int* row_unit = nullptr; // bagging by query: query of each row
  int num_units = 0;             // bagging by query: number of queries
  const uint2* jump = nullptr;   // bagging: state after j + 1 steps = jump[j].x * s + jump[j].y
  int* tile_cnt = nullptr;       // kept rows per tile
  unsigned* tile_sel = nullptr;  // GOSS, 4 words per tile: top threshold bits, key threshold, key mode, multiplier bits
  int* out = nullptr;            // kept rows, ascending
  int* oob = nullptr;            // nullptr, or the rows NOT kept, ascending (out-of-bag score walk)
  int* total = nullptr;          // kept row count
};

inline int SampleTiles(int n) { return (n + kSampleTile - 1) / kSampleTile; }

// per-tile decisions and kept counts
void LaunchSampleCount(const SampleArgs& a, hipStream_t s);
// stable compaction of the kept rows (+ GOSS scaling, + bagging stream advance); writes *total
void LaunchSampleScatter(const SampleArgs& a, hipStream_t s);
// bagging by query: advance the per-1024-query streams past this bag's draws
// (a separate launch: every row tile reads the shared query streams)
void LaunchSampleAdvanceUnits(const SampleArgs& a, hipStream_t s);
// (a^j, c_j) of the reference LCG for j = 1..1024 (host side)
void BuildLcgJumpTable(uint2* out);

}  // namespace device
}  // namespace lgap
