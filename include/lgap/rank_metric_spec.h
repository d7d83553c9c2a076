// Ranking / AUC metrics evaluated where the score lives (the device learner's HBM copy):
// the metric describes itself once (kind, weights, per-query tables the host computes at
// Init) and turns the device's raw sums into its values. Reference metrics:
// binary_metric.hpp:159-268 (AUC, average precision), rank_metric.hpp:86-165 (NDCG@k),
// map_metric.hpp:107-160 (MAP@k), the fork's precision_metric.hpp:16-141 (precision@k).
#pragma once

#include <vector>

#include "lgap/meta.h"

namespace lgap {

struct RankMetricSpec {
  enum Kind { kAUC = 0, kAveragePrecision = 1, kNDCG = 2, kMAP = 3, kPrecision = 4 };
  int kind = -1;
  const void* owner = nullptr;  // the metric instance: device tables are cached per owner
  data_size_t num_data = 0;
  const label_t* label = nullptr;    // host arrays of the metric's dataset (identity checks)
  const label_t* weights = nullptr;  // AUC / AP row weights (nullptr: all 1)
  // query metrics
  data_size_t num_queries = 0;
  const data_size_t* query_boundaries = nullptr;  // [num_queries + 1]
  const label_t* query_weights = nullptr;         // nullptr: all 1
  std::vector<int> eval_at;
  std::vector<double> label_gain;  // NDCG
  std::vector<double> inv_max;     // NDCG [num_queries][eval_at]: 1 / ideal DCG, or -1 (no relevant row)
  std::vector<int> npos;           // MAP [num_queries]: relevant rows
  // The device returns raw sums: AUC / AP {accumulator, positive weight}; query metrics the
  // query-weighted sums per eval_at position. Kept small enough for one pass of the kernels.
  static constexpr int kMaxEvalAt = 32;
};

// auc_mu (reference multiclass_metric.hpp AucMuMetric): for every class pair (i < j) the rows
// of classes i and j, scored by t1 * sum_m v_m score_m (v = cw[i] - cw[j], t1 = v_i - v_j),
// give S_ij = sum over i-rows of w * (j-weight scored below + half the tied j-weight): a
// binary AUC accumulator with class i positive. The device returns S_ij per pair.
struct AucMuSpec {
  const void* owner = nullptr;
  data_size_t num_data = 0;
  const label_t* label = nullptr;
  const label_t* weights = nullptr;
  int num_class = 0;
  const std::vector<data_size_t>* sorted = nullptr;  // rows ordered by class (stable)
  const std::vector<int>* sizes = nullptr;           // rows per class
  const std::vector<std::vector<double>>* cw = nullptr;
  static constexpr int kMaxClass = 64;
};

}  // namespace lgap
